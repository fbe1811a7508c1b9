"""Device Trace2 time at BASELINE configs[2] for several GSA_TRACE_BAND widths (0: every tile recomputed on entry)."""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import gpuseqalign_amd as gsa
from gpuseqalign_amd import formats as F
import bench
sub = bench.subst_blosum62()
eng = gsa.Engine(0)
dev = torch.device("cuda:0")
d = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.int32)).to(dev)
X = F.synthetic_seq(100000, 100); Y = F.mutate_seq(X, 101)
for band in (sys.argv[1:] or ["0", "2048", "4096"]):
    os.environ["GSA_TRACE_BAND"] = band
    geom = gsa.sparse_geometry(len(Y), len(X), 256)
    y, x, s = d(Y), d(X), d(sub)
    hr = torch.empty(geom.hrowElems, dtype=torch.int32, device=dev); hc = torch.empty(geom.hcolElems, dtype=torch.int32, device=dev)
    args = (y.data_ptr(), len(Y), x.data_ptr(), len(X), s.data_ptr(), 25, -11)
    eng.fill_sparse_dev(*args, 256, hr.data_ptr(), hc.data_ptr()); eng.sync()
    ts = []
    for _ in range(3):
        torch.cuda.synchronize(); t = time.perf_counter()
        r = eng.trace_sparse_dev(*args, geom, hr.data_ptr(), hc.data_ptr())
        torch.cuda.synchronize(); ts.append(time.perf_counter() - t)
    print(json.dumps({"band": band, "trace_ms": round(1e3 * min(ts), 2), "cost": r[2], "hash": r[0]}), flush=True)
