"""A/B of score-only variants on the config-5 50k pair (default: GSA_SCORE_BIDI 0 / 1): kernel ms
(HIP events around the whole call) per mode, variants interleaved, median of N calls, scores
compared.  usage: r05_bidi_ab.py [n] [reps] [modes] [variant ...], a variant = ENV=V[,ENV=V...]
with GSA_ prefixes implied, modes a comma list of NW-AG, NW-LG, SW-LG."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gpuseqalign_amd as gsa  # noqa: E402
from gpuseqalign_amd import formats as F  # noqa: E402
from bench import subst_blosum62  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 50000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 7
modes = (sys.argv[3] if len(sys.argv) > 3 else "NW-AG,NW-LG,SW-LG").split(",")
variants = sys.argv[4:] or ["SCORE_BIDI=0", "SCORE_BIDI=1"]
ALL = {"NW-AG": (-11, -1, False), "NW-LG": (-11, -11, False), "SW-LG": (-11, -11, True)}
dev = torch.device("cuda:0")
Y, X = F.synthetic_seq(n, 200), F.synthetic_seq(n, 201)
y, x, s = (torch.from_numpy(np.ascontiguousarray(a, dtype=np.int32)).to(dev) for a in (Y, X, subst_blosum62()))
eng = gsa.Engine(0)
R, C = len(Y) - 1, len(X) - 1
keys = sorted({kv.split("=")[0] for v in variants for kv in v.split(",")})


def setv(v):
    for k in keys:
        os.environ.pop("GSA_" + k, None)
    for kv in v.split(","):
        k, val = kv.split("=")
        os.environ["GSA_" + k] = val


for name in modes:
    go, ge, local = ALL[name]
    run = lambda: eng.score_dev(y.data_ptr(), len(Y), x.data_ptr(), len(X), s.data_ptr(), 25, go, ge, local)
    for v in variants:
        setv(v)
        run()
    ks = {v: [] for v in variants}
    out = {}
    for _ in range(reps):
        for v in variants:
            setv(v)
            r = run()
            ks[v].append(r["kernel_ms"])
            out[v] = (r["score"], r["i_end"], r["j_end"])
    line = [f"{name} n={n}", f"same={len(set(out.values())) == 1}", str(out[variants[0]])]
    for v in variants:
        med = float(np.median(ks[v]))
        line.append(f"{v}: {med:.3f} ms {R * C / med / 1e6:.1f} GCUPS (min {min(ks[v]):.3f})")
    print(" | ".join(line), flush=True)
