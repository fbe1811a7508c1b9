"""A/B of score-only NW from both ends (GSA_SCORE_BIDI 0 / 1) on the config-5 50k pair: kernel ms
(HIP events around the whole call) per mode, interleaved, median of N calls, scores compared."""
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
dev = torch.device("cuda:0")
Y, X = F.synthetic_seq(n, 200), F.synthetic_seq(n, 201)
y, x, s = (torch.from_numpy(np.ascontiguousarray(a, dtype=np.int32)).to(dev) for a in (Y, X, subst_blosum62()))
eng = gsa.Engine(0)
R, C = len(Y) - 1, len(X) - 1
for name, go, ge, local in [("NW-AG", -11, -1, False), ("NW-LG", -11, -11, False), ("SW-LG", -11, -11, True)]:
    res = {}
    for b in ("0", "1"):
        os.environ["GSA_SCORE_BIDI"] = b
        eng.score_dev(y.data_ptr(), len(Y), x.data_ptr(), len(X), s.data_ptr(), 25, go, ge, local)
    ks = {"0": [], "1": []}
    out = {}
    for _ in range(reps):
        for b in ("0", "1"):
            os.environ["GSA_SCORE_BIDI"] = b
            r = eng.score_dev(y.data_ptr(), len(Y), x.data_ptr(), len(X), s.data_ptr(), 25, go, ge, local)
            ks[b].append(r["kernel_ms"])
            out[b] = (r["score"], r["i_end"], r["j_end"])
    line = [name, f"same={out['0'] == out['1']}", str(out["1"])]
    for b in ("0", "1"):
        med = float(np.median(ks[b]))
        line.append(f"bidi={b}: {med:.3f} ms {R * C / med / 1e6:.1f} GCUPS (min {min(ks[b]):.3f})")
    print(" | ".join(line), flush=True)
