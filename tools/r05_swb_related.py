"""SW-LG / SW-AG score-only on 50k pairs whose best alignment crosses the split (a related pair) and
does not (a random pair): kernel ms (score_dev, HIP events) one direction (GSA_SCORE_BIDI_SW=0) and
from both ends (default; a crossing pair then runs again in one direction); 3 calls each after 1
untimed."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import gpuseqalign_amd as gsa  # noqa: E402
from gpuseqalign_amd import formats as F  # noqa: E402
from tests._data import Golden  # noqa: E402

g = Golden()
sub = np.ascontiguousarray(g.blosum62, dtype=np.int32)
eng = gsa.Engine(0)
dev = torch.device("cuda:0")
s = torch.from_numpy(sub).to(dev)
n = int(round(np.sqrt(sub.size)))
x = F.synthetic_seq(50000, 500)
yr = F.mutate_seq(x, 501)
yr = yr[:len(yr) - (len(yr) - 1) % 2]
rng = np.random.default_rng(7)
yrand = np.concatenate([[0], rng.integers(0, 20, 50000)]).astype(np.int32)
xrand = np.concatenate([[0], rng.integers(0, 20, 50000)]).astype(np.int32)
for name, (Y, X) in (("related", (yr, x)), ("random", (yrand, xrand))):
    ty, tx = torch.from_numpy(np.ascontiguousarray(Y, dtype=np.int32)).to(dev), torch.from_numpy(np.ascontiguousarray(X, dtype=np.int32)).to(dev)
    for go, ge in ((-11, -11), (-11, -1)):
        line = []
        for label, env in (("one direction", {"GSA_SCORE_BIDI_SW": "0"}), ("both ends", {}),
                           ("both ends, whole rerun", {"GSA_BIDI_SW_CONT": "0"})):
            for k in ("GSA_SCORE_BIDI_SW", "GSA_BIDI_SW_CONT"):
                os.environ.pop(k, None)
            os.environ.update(env)
            res = None
            ms = []
            for it in range(4):
                r = eng.score_dev(ty.data_ptr(), len(Y), tx.data_ptr(), len(X), s.data_ptr(), n, go, ge, True)
                if it:
                    ms.append(r["kernel_ms"])
                res = (r["score"], r["i_end"], r["j_end"])
            line.append(f"{label} {min(ms):.3f} ms {res}")
        print(f"{name} {len(Y) - 1}x{len(X) - 1} SW {go}/{ge}: " + " | ".join(line), flush=True)
