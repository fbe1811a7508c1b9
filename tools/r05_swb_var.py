"""Random 50k SW-LG / SW-AG score-only: kernel ms of 8 calls each from both ends (default) and in one
direction (GSA_SCORE_BIDI_SW=0), interleaved."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import gpuseqalign_amd as gsa  # noqa: E402
from tests._data import Golden  # noqa: E402

sub = np.ascontiguousarray(Golden().blosum62, dtype=np.int32)
n = int(round(np.sqrt(sub.size)))
eng = gsa.Engine(0)
dev = torch.device("cuda:0")
s = torch.from_numpy(sub).to(dev)
rng = np.random.default_rng(7)
Y = torch.from_numpy(np.concatenate([[0], rng.integers(0, 20, 50000)]).astype(np.int32)).to(dev)
X = torch.from_numpy(np.concatenate([[0], rng.integers(0, 20, 50000)]).astype(np.int32)).to(dev)
variants = (("both ends", {}), ("one direction", {"GSA_SCORE_BIDI_SW": "0"}))
for go, ge in ((-11, -11), (-11, -1)):
    res = {v: [] for v, _ in variants}
    for it in range(9):
        for v, env in variants:
            for k in ("GSA_SCORE_BIDI_SW",):
                os.environ.pop(k, None)
            os.environ.update(env)
            r = eng.score_dev(Y.data_ptr(), 50001, X.data_ptr(), 50001, s.data_ptr(), n, go, ge, True)
            if it:
                res[v].append(round(r["kernel_ms"], 3))
    for v in res:
        print(f"SW {go}/{ge} {v}: median {np.median(res[v]):.3f} ms  {res[v]}", flush=True)
