"""Diagnostic: run one fill on the stamp build (libgsa_stamp.so) and summarise per-wave
block timings (s_memtime cycles): sweep, post-sweep work, barrier wait."""
import os, sys, ctypes, argparse
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["GSA_LIB"] = os.path.join(ROOT, "gpuseqalign_amd", "libgsa_stamp.so")
sys.path.insert(0, ROOT)
import numpy as np
import gpuseqalign_amd as gsa
from tests._data import Golden, random_pair

ap = argparse.ArgumentParser()
ap.add_argument("--R", type=int, default=256)
ap.add_argument("--C", type=int, default=20000)
ap.add_argument("--mode", default="sparse")
a = ap.parse_args()
G = Golden()
eng = gsa.Engine(0)
Y, X = random_pair(a.R, a.C, 3)
for _ in range(2):
    if a.mode == "sparse":
        r = eng.align_sparse(Y, X, G.blosum62, -11, tileBx=256)
    else:
        r = eng.align_full(Y, X, G.blosum62, -11)
print("laps", r.laps)
L = gsa.lib()
L.gsa_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]
n = 16 * 256 * 4
buf = (ctypes.c_uint64 * n)()
assert L.gsa_debug_stamps(eng._h, buf, n) == 0
st = np.frombuffer(buf, dtype=np.uint64).reshape(16, 256, 4).astype(np.int64)
for w in range(8):
    s = st[w]
    if s[:, 0].max() == 0:
        continue
    idx = np.where((s[:, 0] > 0) & (s[:, 3] > 0))[0]
    idx = idx[(idx > 20) & (idx < 250)]
    if len(idx) < 3:
        continue
    blk = np.diff(s[idx, 0])
    wait, flags, comp = s[idx, 1] - s[idx, 0], s[idx, 2] - s[idx, 1], s[idx, 3] - s[idx, 2]
    print(f"wave {w}: block {np.median(blk):.0f} cyc = wait {np.median(wait):.0f} + halo/flags {np.median(flags):.0f}"
          f" + compute {np.median(comp):.0f} (+ tail {np.median(blk) - np.median(wait+flags+comp):.0f})  n={len(idx)}")
    print("   blocks", blk[:10].tolist(), " wait", wait[:10].tolist())
