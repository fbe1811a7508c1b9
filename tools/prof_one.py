"""Run one fill configuration a few times (for rocprofv3 sessions).
--config3: the bench's headline pair (BASELINE configs[2], related 100k pair, seeds 100/101)."""
import os, sys, argparse, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import gpuseqalign_amd as gsa
from tools.gpu_perf import run

ap = argparse.ArgumentParser()
ap.add_argument("--R", type=int, default=252)
ap.add_argument("--C", type=int, default=20000)
ap.add_argument("--mode", default="sparse")
ap.add_argument("--tileBx", type=int, default=256)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--config3", action="store_true")
a = ap.parse_args()
eng = gsa.Engine(0)
if a.config3:
    import bench
    Y, X = bench.config3_pair()
    dev = torch.device("cuda:0")
    y, x, s = (torch.from_numpy(np.ascontiguousarray(v, dtype=np.int32)).to(dev) for v in (Y, X, bench.subst_blosum62()))
    g = gsa.sparse_geometry(len(Y), len(X), a.tileBx)
    hr = torch.empty(g.hrowElems, dtype=torch.int32, device=dev)
    hc = torch.empty(g.hcolElems, dtype=torch.int32, device=dev)
    for _ in range(a.reps):
        eng.fill_sparse_dev(y.data_ptr(), len(Y), x.data_ptr(), len(X), s.data_ptr(), 25, -11, a.tileBx,
                            hr.data_ptr(), hc.data_ptr())
    eng.sync()
    print(json.dumps({"R": len(Y) - 1, "C": len(X) - 1, "reps": a.reps}))
else:
    print(run(eng, a.R, a.C, a.mode, a.tileBx, reps=a.reps))
