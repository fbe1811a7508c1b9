"""Diagnostic (stamp build): the per-pair kernel arguments each ticket's workgroup saw."""
import os, sys, ctypes
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["GSA_LIB"] = os.path.join(ROOT, "gpuseqalign_amd", "libgsa_stamp.so")
sys.path.insert(0, ROOT)
import numpy as np
import gpuseqalign_amd as gsa
from tests._data import Golden, random_pair
G = Golden()
R, C = int(sys.argv[1]), int(sys.argv[2])
Y, X = random_pair(R, C, 3)
eng = gsa.Engine(0)
try:
    r = eng.align_sparse(Y, X, G.blosum62, -11, tileBx=64)
    print("ok cost", r.align_cost)
except Exception as e:
    print("error", e)
L = gsa.lib()
L.gsa_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]
n = 16 * 256 * 4
buf = (ctypes.c_uint64 * n)()
L.gsa_debug_stamps(eng._h, buf, n)
st = np.frombuffer(buf, dtype=np.uint64)[16000 - 64 * 6:16000].reshape(64, 6)
g = gsa.sparse_geometry(R + 1, C + 1, 64)
top = np.frombuffer(buf, dtype=np.uint64)[16100:16100 + 64].reshape(8, 8)
for b in range(3):
    print("wg", b, "mark %x tkg %d nTT %d pairs %x nPairs %d err %d ticket %x" % tuple(int(v) for v in top[b][:7]))
print("expect R C", R, C, "Cp", g.tileHdrMatCols * 64, "trows tcols", g.tileHdrMatRows, g.tileHdrMatCols)
sw = np.frombuffer(buf, dtype=np.uint64)[16200:16200 + 128].reshape(16, 8)
for i in range(8):
    w = [int(v) for v in sw[i]]
    if w[0] == 0:
        continue
    print("strip tk", i // 4, "w", i % 4, "hcol %x" % w[1], "R", w[2] >> 32, "C", w[2] & 0xffffffff, "Cp", w[3] >> 32,
          "nT", w[3] & 0xffffffff, "trows", w[4] >> 32, "tcols", w[4] & 0xffffffff, "tBx", w[5] >> 32, "r0", w[5] & 0xffffffff,
          "seqY %x gran %x" % (w[6], w[7]))
for t in range(4):
    w = [int(v) for v in st[t]]
    if w[0] == 0 and w[2] == 0:
        continue
    print("ticket", t, "hcol %x hrow %x" % (w[0], w[1]), "R", w[2] >> 32, "C", w[2] & 0xffffffff, "Cp", w[3] >> 32,
          "nT", w[3] & 0xffffffff, "trows", w[4] >> 32, "tcols", w[4] & 0xffffffff, "tBx", w[5] >> 32, "tk", w[5] & 0xffffffff)
