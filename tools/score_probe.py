"""Decompose the score-only kernel's time: one tile row (per-wave panel time), one panel per
tile row (hop latency + panel time), and the square case."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import gpuseqalign_amd as gsa
from gpuseqalign_amd import formats as F
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sub = F.read_subst_json(os.path.join(ROOT, "tests", "golden", "resrc", "subst.json")).matrix("blosum62")
eng = gsa.Engine(0)
d = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.int32)).to("cuda:0")
s = d(sub)
for R, C in [(64, 50000), (50000, 64), (6400, 6400), (50000, 50000), (50000, 1280)]:
    Y, X = F.synthetic_seq(R, 200), F.synthetic_seq(C, 201)
    y, x = d(Y), d(X)
    ks = [eng.score_dev(y.data_ptr(), len(Y), x.data_ptr(), len(X), s.data_ptr(), 25, -11, -1, False)["kernel_ms"]
          for _ in range(4)]
    ms = float(np.median(ks[1:]))
    nTR, nP = (R + 63) // 64, (C + 63) // 64
    print(json.dumps({"R": R, "C": C, "nTR": nTR, "nP": nP, "ms": round(ms, 3),
                      "us_per_panel_if_serial_panels": round(1e3 * ms / nP, 2) if nTR == 1 else None,
                      "us_per_hop_if_serial_rows": round(1e3 * ms / nTR, 2) if nP == 1 else None,
                      "gcups": round(R * C / ms / 1e6, 1)}), flush=True)
