"""BASELINE configs[4]: score-only SW-LG and NW-AG (gapo -11, gape -1) on a 50k x 50k random
pair (seeds 200/201), GPU kernel time (hipEvent, device-resident inputs) and the CPU baseline
(oracle/score_oracle.c tiled OpenMP wavefront, blocksz 256, cpu4-mt-diagrow shape) on the
box's host cores.  One JSON line per configuration."""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import gpuseqalign_amd as gsa
from gpuseqalign_amd import formats as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sub = F.read_subst_json(os.path.join(ROOT, "tests", "golden", "resrc", "subst.json")).matrix("blosum62")
eng = gsa.Engine(0)
dev = torch.device("cuda:0")
d = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.int32)).to(dev)
threads = int(os.environ.get("CPU_THREADS", "16"))
for n in [int(x) for x in (sys.argv[1:] or ["50000"])]:
    Y, X = F.synthetic_seq(n, 200), F.synthetic_seq(n, 201)
    y, x, s = d(Y), d(X), d(sub)
    for name, go, ge, local in [("SW-LG", -11, -11, True), ("NW-AG", -11, -1, False), ("SW-AG", -11, -1, True),
                                ("NW-LG", -11, -11, False)]:
        ks = []
        for _ in range(4):
            r = eng.score_dev(y.data_ptr(), len(Y), x.data_ptr(), len(X), s.data_ptr(), 25, go, ge, local)
            ks.append(r["kernel_ms"])
        kms = float(np.median(ks[1:]))
        line = {"config": name, "R": n, "C": n, "gapo": go, "gape": ge, "score": r["score"],
                "end": [r["i_end"], r["j_end"]], "kernel_ms": round(kms, 3), "gcups": round(n * n / kms / 1e6, 1)}
        if n <= 50000 and name in ("SW-LG", "NW-AG") and not os.environ.get("NO_CPU"):
            import oracle
            m = 12000  # bounded CPU sample: a 12k x 12k prefix of the same pair
            t = time.perf_counter()
            oracle.score_ag(Y[:m + 1], X[:m + 1], sub, go, ge, local, mt=True, blocksz=256, nthreads=threads)
            cs = time.perf_counter() - t
            line["cpu_baseline"] = {"gcups": round(m * m / cs / 1e9, 3), "threads": threads,
                                    "kind": "port (score_oracle.c tiled OpenMP wavefront)",
                                    "sample": f"{m}x{m} prefix of the same pair"}
        print(json.dumps(line), flush=True)
