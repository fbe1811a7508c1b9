"""Diagnostic: one full fill on a stamp build of the lane kernel (GSA_LIB), per-wave block
timings of ticket 0 (s_memtime cycles, blocks 100..355): wait, compute, stores."""
import os, sys, ctypes
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
import gpuseqalign_amd as gsa
from tests._data import Golden, random_pair
R = int(sys.argv[1]) if len(sys.argv) > 1 else 64
C = int(sys.argv[2]) if len(sys.argv) > 2 else 10000
G = Golden()
eng = gsa.Engine(0)
Y, X = random_pair(R, C, 3)
for _ in range(2):
    r = eng.align_full(Y, X, G.blosum62, -11)
print("R", R, "C", C, "laps", r.laps)
L = gsa.lib()
L.gsa_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]
n = 16 * 256 * 4
buf = (ctypes.c_uint64 * n)()
assert L.gsa_debug_stamps(eng._h, buf, n) == 0
st = np.frombuffer(buf, dtype=np.uint64).reshape(16, 256, 4).astype(np.int64)
for w in range(16):
    s = st[w]
    if s[:, 0].max() == 0:
        continue
    blk = np.diff(s[:, 0])
    wait, comp, sto = s[:, 1] - s[:, 0], s[:, 2] - s[:, 1], s[:, 3] - s[:, 2]
    tail = blk - (wait + comp + sto)[:-1]
    print(f"wave {w}: block med {np.median(blk):.0f} mean {blk.mean():.0f} = wait {np.median(wait):.0f} + compute {np.median(comp):.0f}"
          f" + ring/stores {np.median(sto):.0f} + tail {np.median(tail):.0f}")
    print("   blocks", blk[:24].tolist())
    print("   wait  ", wait[:24].tolist())
    print("   comp  ", comp[:24].tolist())
