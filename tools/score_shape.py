"""Score-only kernel time on R x C random pairs (seeds 200/201), per mode: the steady per-block
rate (one ticket, R = 1024) against the whole pair.  Diagnostics only.
usage: python tools/score_shape.py 1024x50000 50000x50000 [MODES=NW-AG,SW-LG,NW-LG,SW-AG]"""
import json, os, sys
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
modes = {"SW-LG": (-11, -11, True), "NW-AG": (-11, -1, False), "SW-AG": (-11, -1, True), "NW-LG": (-11, -11, False)}
want = os.environ.get("MODES", "NW-AG,SW-LG").split(",")
for shp in sys.argv[1:]:
    R, C = map(int, shp.split("x"))
    Y, X = F.synthetic_seq(R, 200), F.synthetic_seq(C, 201)
    y, x, s = d(Y), d(X), d(sub)
    for name in want:
        go, ge, local = modes[name]
        ks = [eng.score_dev(y.data_ptr(), len(Y), x.data_ptr(), len(X), s.data_ptr(), 25, go, ge, local) for _ in range(5)]
        kms = float(np.median([r["kernel_ms"] for r in ks[1:]]))
        r = ks[-1]
        print(json.dumps({"mode": name, "R": R, "C": C, "score": r["score"], "end": [r["i_end"], r["j_end"]],
                          "kernel_ms": round(kms, 4), "gcups": round(R * C / kms / 1e6, 1)}), flush=True)
