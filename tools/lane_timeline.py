"""Diagnostic: per-strip block-start timeline of the lane kernel (stamp build, GSA_LIB):
lag of strip k behind strip k-1 at equal block index, in cycles and in steps."""
import os, sys, ctypes
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
import gpuseqalign_amd as gsa
from tests._data import Golden, random_pair
R = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
C = int(sys.argv[2]) if len(sys.argv) > 2 else 10000
G = Golden()
eng = gsa.Engine(0)
Y, X = random_pair(R, C, 3)
for _ in range(2):
    r = eng.align_full(Y, X, G.blosum62, -11)
print("R", R, "C", C, "kernel ms", r.laps.get("calc_kernel_ms"))
L = gsa.lib()
L.gsa_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]
n = 16 * 160
buf = (ctypes.c_uint64 * n)()
assert L.gsa_debug_stamps(eng._h, buf, n) == 0
st = np.frombuffer(buf, dtype=np.uint64).reshape(16, 160).astype(np.int64)
ns = int(os.environ.get("GSA_LANE_NS", "2"))
rows = [(tk, w) for tk in range(8) for w in range(min(ns, 2))]
t0 = st[st > 0].min()
prev = None
for tk, w in rows:
    s = st[tk * 2 + w]
    ok = s > 0
    if ok.sum() < 4:
        continue
    idx = np.where(ok)[0]
    per8 = np.diff(s[idx]) * 24.0 / np.diff(idx) / 8 / 16  # cycles per step (100 MHz ticks x 24 @2.4 GHz)
    line = f"tk {tk} w {w}: start {s[idx[0]] - t0:8d}  step cyc med {np.median(per8):6.1f} (first {per8[:3].round(1).tolist()} last {per8[-3:].round(1).tolist()})"
    if prev is not None:
        both = ok & (prev > 0)
        lag = (s[both] - prev[both]) * 24
        line += f"  lag vs prev: med {np.median(lag):7.0f} cyc, first {lag[:3].tolist()}, last {lag[-3:].tolist()}"
    print(line)
    prev = s
