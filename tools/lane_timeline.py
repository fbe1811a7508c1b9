"""Diagnostic: per-strip block-start timeline of the lane kernel (stamp build, GSA_LIB), from
s_memrealtime stamps (100 MHz, one clock for all XCDs; x24 = cycles at 2.4 GHz): lag of each
strip behind the previous one at equal block index, and the inter-workgroup link of tickets
0 -> 1 (drain store, feed receipt) against the producer's block starts."""
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
n = 3200
buf = (ctypes.c_uint64 * n)()
assert L.gsa_debug_stamps(eng._h, buf, n) == 0
allst = np.frombuffer(buf, dtype=np.uint64).astype(np.int64)
xcc = allst[3100:3200]
st = allst[:2560].reshape(16, 160)
ns = int(os.environ.get("GSA_LANE_NS", "2"))
stride = int(os.environ.get("STRIDE", "1"))  # the stamp build's GSA_STAMP_STRIDE
rows = [(sidx * stride // ns, sidx * stride % ns) for sidx in range(16)]
t0 = st[st > 0].min()
prev = None
for i, (tk, w) in enumerate(rows):
    s = st[i]
    ok = s > 0
    if ok.sum() < 4:
        continue
    idx = np.where(ok)[0]
    per8 = np.diff(s[idx]) * 24.0 / np.diff(idx) / 8 / 16  # cycles per step
    line = f"tk {tk} (xcd {xcc[tk]}) w {w}: start {s[idx[0]] - t0:8d}  step cyc med {np.median(per8):6.1f} (first {per8[:3].round(1).tolist()} last {per8[-3:].round(1).tolist()})"
    if prev is not None:
        both = ok & (prev > 0)
        lag = (s[both] - prev[both]) * 24
        line += f"  lag vs prev: med {np.median(lag):7.0f} cyc, first {lag[:3].tolist()}, last {lag[-3:].tolist()}"
    print(line)
    prev = s
# link ticket 0 -> 1.  Column 64k is written by the producer (ticket 0's last strip) in block
# 4k+4 and computed by the consumer (ticket 1, strip 0) in block 4k.  Block starts are stamped
# every 8 blocks; the others are interpolated.
if stride != 1:
    sys.exit(0)
drain = allst[2560:2760]
feed = allst[2800:3000]
prod = st[ns - 1].astype(float)
cons = st[ns].astype(float)
def at(s, blk):
    i = blk / 8.0
    lo = int(np.floor(i))
    if lo + 1 >= len(s) or s[lo] == 0 or s[lo + 1] == 0:
        return None
    return s[lo] + (s[lo + 1] - s[lo]) * (i - lo)
print("link ticket 0 -> 1 (cycles after the start of the producer block that writes the column):")
for k in range(2, 150, 8):
    p0, c0 = at(prod, 4 * k + 4), at(cons, 4 * k)
    if p0 is None or c0 is None or drain[k] == 0 or feed[k] == 0:
        continue
    print(f"  col {64 * k:5d}: drained +{(drain[k] - p0) * 24:7.0f}  fed +{(feed[k] - p0) * 24:7.0f}  consumer block +{(c0 - p0) * 24:7.0f}")
