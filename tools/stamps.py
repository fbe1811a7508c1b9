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
ap.add_argument("--R", type=int, default=252)
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
for w in range(10):
    s = st[w]
    if s[:, 0].max() == 0:
        continue
    valid = (s[:, 0] > 0) & (s[:, 2] > 0)
    idx = np.where(valid)[0]
    idx = idx[(idx > 40) & (idx < 250)]
    blk = np.diff(s[idx, 0])
    sweep = (s[idx, 1] - s[idx, 0]) if s[idx, 1].max() > 0 else np.zeros(len(idx))
    post = (s[idx, 2] - s[idx, 1]) if s[idx, 1].max() > 0 else (s[idx, 2] - s[idx, 0])
    wait = s[idx[:-1] + 1, 0] - s[idx[:-1], 2]
    print(f"wave {w}: block {np.median(blk):.0f} cyc, sweep {np.median(sweep):.0f}, post {np.median(post):.0f}, barrier wait {np.median(wait):.0f}  (n={len(idx)})")
    print("   sample block lengths", blk[:12].tolist())
