"""Per-block stamps of the K-rows sparse fill (GSA_LIB = a tools/patches/krow_stamps2.py build): block
period, wait at the progress check with the condition that failed, work, lag between strips.
Diagnostics only.  usage: GSA_LIB=... python tools/kr_stamps2.py [RxC|config3]"""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import gpuseqalign_amd as gsa
import bench
from gpuseqalign_amd import formats as F

shape = sys.argv[1] if len(sys.argv) > 1 else "config3"
if shape == "config3":
    Y, X = bench.config3_pair()
else:
    r, c = map(int, shape.split("x"))
    Y, X = F.synthetic_seq(r, 11), F.synthetic_seq(c, 12)
sub = bench.subst_blosum62()
dev = torch.device("cuda:0")
y, x, s = (torch.from_numpy(np.ascontiguousarray(v, dtype=np.int32)).to(dev) for v in (Y, X, sub))
g = gsa.sparse_geometry(len(Y), len(X), 256)
hr = torch.empty(g.hrowElems, dtype=torch.int32, device=dev)
hc = torch.empty(g.hcolElems, dtype=torch.int32, device=dev)
eng = gsa.Engine(0)
st = torch.cuda.current_stream()
for _ in range(3):
    eng.fill_sparse_dev(y.data_ptr(), len(Y), x.data_ptr(), len(X), s.data_ptr(), 25, -11, 256, hr.data_ptr(),
                        hc.data_ptr(), st.cuda_stream)
    eng.sync(st.cuda_stream)
L = ctypes.CDLL(os.environ["GSA_LIB"])
a = np.zeros((32, 6400, 4), np.uint64)
assert L.gsa_dbg_kst2(a.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(a.nbytes)) == 0
a = a.astype(np.int64)
C = len(X) - 1
NB = min(6400, (C + 65 + 15) // 16)
ns = min(32, (len(Y) - 1 + 255) // 256)
t0 = a[:ns, :NB, 0]; t1 = a[:ns, :NB, 1]; t2 = a[:ns, :NB, 2]; why = a[:ns, :NB, 3]
lo, hi = 8, NB - 8
print(f"shape {shape}: NB {NB}, strips {ns}")
for w in range(ns):
    per = np.diff(t1[w, lo:hi]); wait = (t1 - t0)[w, lo:hi]; work = (t2 - t1)[w, lo:hi]; wy = why[w, lo:hi]
    rest = t0[w, lo + 1:hi] - t2[w, lo:hi - 1]
    line = (f"strip {w:2d}: period {np.median(per):5.0f}/{per.mean():5.0f} | wait {np.median(wait):4.0f}/{wait.mean():5.0f} "
            f"| work {np.median(work):5.0f} | after {np.median(rest):4.0f}/{rest.mean():4.0f} | fail prog {np.mean(wy & 1 > 0):.2f} "
            f"cons {np.mean(wy & 2 > 0):.2f} xo {np.mean(wy & 4 > 0):.2f}")
    if w > 0:
        lag = (t1[w, lo:hi] - t1[w - 1, lo:hi])
        line += f" | lag {np.median(lag):6.0f} ({np.median(lag) / np.median(per):.2f} blk)"
    print(line)
w = min(5, ns - 1)
ph = (np.arange(lo, hi) % 16)
for name, arr in [("work", (t2 - t1)[w, lo:hi]), ("wait", (t1 - t0)[w, lo:hi]),
                  ("after", np.concatenate([t0[w, lo + 1:hi] - t2[w, lo:hi - 1], [0]]))]:
    print(f"{name} by b%16 (strip {w}):", " ".join(f"{np.median(arr[ph == k]):.0f}" for k in range(16)))
