"""A/B of the sparse single-pair kernels on the bench's headline pair (BASELINE configs[2]):
GSA_SPARSE_KERNEL / GSA_PAIR2_NS are read per launch, so one process times every variant.
Each variant: warm-up, then `reps` fills timed with HIP events on the launch stream; the
align_cost of the last fill is checked against tests/golden/config3_100k.json."""
import argparse, json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import gpuseqalign_amd as gsa
import bench

ap = argparse.ArgumentParser()
ap.add_argument("--variants", default="strip:4,krow:4:4,krow:4:2,krow:2:4")
ap.add_argument("--reps", type=int, default=10)
ap.add_argument("--tileBx", type=int, default=256)
ap.add_argument("--shapes", default="", help="RxC,... (random pairs) or config3 (the headline pair); default config3")
a = ap.parse_args()
from gpuseqalign_amd import formats as F
sub = bench.subst_blosum62()
shapes = [None if t == "config3" else tuple(map(int, t.split("x"))) for t in a.shapes.split(",") if t] or [None]
for shp in shapes:
  if shp:
    Y, X = F.synthetic_seq(shp[0], 11), F.synthetic_seq(shp[1], 12)
  else:
    Y, X = bench.config3_pair()
  gold = json.load(open(os.path.join(bench.ROOT, "tests", "golden", "config3_100k.json")))["pairs"]["related"]["align_cost"]
  dev = torch.device("cuda:0")
  y, x, s = (torch.from_numpy(np.ascontiguousarray(v, dtype=np.int32)).to(dev) for v in (Y, X, sub))
  g = gsa.sparse_geometry(len(Y), len(X), a.tileBx)
  hr = torch.empty(g.hrowElems, dtype=torch.int32, device=dev)
  hc = torch.empty(g.hcolElems, dtype=torch.int32, device=dev)
  eng = gsa.Engine(0)
  st = torch.cuda.current_stream()
  R, C = len(Y) - 1, len(X) - 1
  for v in a.variants.split(","):
      parts = v.split(":")  # kernel:ns[:k]
      os.environ["GSA_SPARSE_KERNEL"] = parts[0]
      os.environ["GSA_PAIR2_NS"] = parts[1]
      os.environ["GSA_KROW_NS"] = parts[1]
      if len(parts) > 2:
          os.environ["GSA_KROW_K"] = parts[2]
      fn = lambda: eng.fill_sparse_dev(y.data_ptr(), len(Y), x.data_ptr(), len(X), s.data_ptr(), 25, -11, a.tileBx,
                                       hr.data_ptr(), hc.data_ptr(), st.cuda_stream)
      fn(); eng.sync(st.cuda_stream)
      ts = []
      for _ in range(a.reps):
          e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
          e0.record(st); fn(); e1.record(st)
          eng.sync(st.cuda_stream)
          ts.append(e0.elapsed_time(e1))
      last = g.tileHdrMatRows * g.tileHdrMatCols - 1
      hrn = np.zeros(g.hrowElems, np.int32); hcn = np.zeros(g.hcolElems, np.int32)
      hrn[last * g.tileHrowLen:] = hr[last * g.tileHrowLen:].cpu().numpy()
      hcn[last * g.tileHcolLen:] = hc[last * g.tileHcolLen:].cpu().numpy()
      cost = gsa.sparse_align_cost(gsa.SparseResult(hrn, hcn, g, 0, {}), Y, X, sub, -11)
      ms = float(np.median(ts))
      print(json.dumps({"variant": v, "R": R, "C": C, "tileBx": a.tileBx, "ms_median": round(ms, 4),
                        "ms_min": round(min(ts), 4), "gcups": round(R * C / ms / 1e6, 1), "align_cost": cost,
                        "golden": gold if not shp else None}), flush=True)
