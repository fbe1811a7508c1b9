"""Diagnostic: per-ticket (super-strip) timeline from the stamp build (libgsa_stamp.so):
when each super-strip's first strip got its profile, became ready (row above available),
its last strip finished, and when its loader fed the first granule chunk."""
import os, sys, ctypes, argparse
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["GSA_LIB"] = os.path.join(ROOT, "gpuseqalign_amd", "libgsa_stamp.so")
sys.path.insert(0, ROOT)
import numpy as np
import gpuseqalign_amd as gsa
from tests._data import Golden, random_pair

ap = argparse.ArgumentParser()
ap.add_argument("--R", type=int, default=10000)
ap.add_argument("--C", type=int, default=10000)
ap.add_argument("--mode", default="full")
ap.add_argument("--ghz", type=float, default=0.1)  # s_memrealtime: 100 MHz
a = ap.parse_args()
G = Golden()
eng = gsa.Engine(0)
Y, X = random_pair(a.R, a.C, 3)
for _ in range(2):
    r = eng.align_sparse(Y, X, G.blosum62, -11, tileBx=256) if a.mode == "sparse" else eng.align_full(Y, X, G.blosum62, -11)
print("kernel ms", r.laps["calc_kernel_ms"])
L = gsa.lib()
L.gsa_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]
n = 16 * 256 * 4
buf = (ctypes.c_uint64 * n)()
assert L.gsa_debug_stamps(eng._h, buf, n) == 0
st = np.frombuffer(buf, dtype=np.uint64)[8192:].reshape(-1, 4).astype(np.int64)
nt = int((st[:, 0] > 0).sum())
st = st[:nt]
base = st[:, 0].min()
us = lambda v: (v - base) / (a.ghz * 1e3) if v > 0 else float("nan")
print("tk   profile   ready   granule0   end    (us)   ready-prev_ready")
prev = None
for tk in range(nt):
    t = [us(v) for v in st[tk]]
    d = t[1] - prev if prev is not None else 0.0
    print(f"{tk:3d} {t[0]:8.1f} {t[1]:8.1f} {t[3]:8.1f} {t[2]:8.1f}   {d:7.2f}")
    prev = t[1]
