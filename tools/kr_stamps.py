"""Diagnostic: per-block timings of the K-rows strips (stamp build tools/build_stamp_lib.sh: GSA_LIB=.../libgsa_p2stamp.so,
nw_krow.hip GSA_KRSTAMP).  One R x C random sparse fill; for strips 0..7 (tickets 0, 1) and
blocks 64..319: block period, wait at block start, 16 steps, capture pick, and the rest."""
import ctypes, os, sys, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
import torch
import gpuseqalign_amd as gsa
from gpuseqalign_amd import formats as F
import bench
R = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
C = int(sys.argv[2]) if len(sys.argv) > 2 else 100000
tBx = int(sys.argv[3]) if len(sys.argv) > 3 else 256
Y, X = F.synthetic_seq(R, 11), F.synthetic_seq(C, 12)
sub = bench.subst_blosum62()
dev = torch.device("cuda:0")
y, x, s = (torch.from_numpy(np.ascontiguousarray(v, dtype=np.int32)).to(dev) for v in (Y, X, sub))
g = gsa.sparse_geometry(len(Y), len(X), tBx)
hr = torch.empty(g.hrowElems, dtype=torch.int32, device=dev)
hc = torch.empty(g.hcolElems, dtype=torch.int32, device=dev)
eng = gsa.Engine(0)
for _ in range(3):
    eng.fill_sparse_dev(y.data_ptr(), len(Y), x.data_ptr(), len(X), s.data_ptr(), 25, -11, tBx, hr.data_ptr(), hc.data_ptr())
    eng.sync()
L = gsa.lib()
L.gsa_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]
n = 16 * 256 * 4
buf = (ctypes.c_uint64 * n)()
assert L.gsa_debug_stamps(eng._h, buf, n) == 0
st = np.frombuffer(buf, dtype=np.uint64).astype(np.int64).reshape(16, 256, 4)
for w in range(8):
    S = st[w]
    if S[:, 0].max() == 0:
        continue
    per = np.diff(S[:, 0])
    wait, steps, cap = S[:, 1] - S[:, 0], S[:, 2] - S[:, 1], S[:, 3] - S[:, 2]
    rest = S[1:, 0] - S[:-1, 3]
    capb = cap > 40
    print(f"strip {w}: period med {np.median(per):.0f} mean {per.mean():.0f} | wait med {np.median(wait):.0f} mean {wait.mean():.0f}"
          f" | steps med {np.median(steps):.0f} | pick med(cap blocks) {np.median(cap[capb]) if capb.any() else 0:.0f} n={capb.sum()}"
          f" | rest med {np.median(rest):.0f} | lag vs strip above at block 64: {S[0,0] - st[w-1][0,0] if w else 0}")
    if w in (0, 3, 4):
        print("   period", per[:32].tolist())
        print("   wait  ", wait[:32].tolist())
        print("   steps ", steps[:32].tolist())
        print("   pick  ", cap[:32].tolist())
