"""Per-block stamps of the K-rows sparse fill (GSA_LIB = a tools/patches/krow_stamps.py build):
block period, wait at the progress check, work, lag between consecutive strips, and the
detection latency (start of strip w's block b minus strip w-1's hand-off publish of block b+4,
the earliest moment it could start).  Diagnostics only.  usage: GSA_LIB=... python tools/kr_stamps.py [RxC|config3]"""
import ctypes, json, os, sys
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
a = np.zeros((32, 6400, 3), np.uint64)
assert L.gsa_dbg_kst(a.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(a.nbytes)) == 0
a = a.astype(np.int64)
C = len(X) - 1
NB = (C + 65 + 15) // 16
ns = min(32, (len(Y) - 1 + 255) // 256)
t0 = a[:ns, :NB, 0]; t1 = a[:ns, :NB, 1]; t2 = a[:ns, :NB, 2]
base = t0[0, 0]
lo, hi = 8, NB - 8
print(f"shape {shape}: NB {NB}, strips {ns}")
for w in range(ns):
    per = np.diff(t1[w, lo:hi]); wait = (t1 - t0)[w, lo:hi]; work = (t2 - t1)[w, lo:hi]
    line = (f"strip {w:2d}: period med {np.median(per):6.0f} mean {per.mean():6.0f} | wait med {np.median(wait):5.0f} "
            f"mean {wait.mean():6.0f} frac>300 {np.mean(wait > 300):.2f} | work med {np.median(work):5.0f} mean {work.mean():6.0f}")
    if w > 0:
        lag = (t1[w, lo:hi] - t1[w - 1, lo:hi])
        det = t1[w, lo:hi - 4] - t2[w - 1, lo + 4:hi]
        line += (f" | lag med {np.median(lag):6.0f} ({np.median(lag) / np.median(per):.2f} blk) | det med {np.median(det):6.0f} "
                 f"p10 {np.percentile(det, 10):6.0f} p90 {np.percentile(det, 90):6.0f}")
    print(line)
# work by block phase (tile boundaries every tBx/16 = 16 blocks)
w = min(5, ns - 1)
work = (t2 - t1)[w, lo:hi]
ph = (np.arange(lo, hi) % 16)
print(f"work by b%16 (strip {w}):", " ".join(f"{np.median(work[ph == k]):.0f}" for k in range(16)))
wait = (t1 - t0)[w, lo:hi]
print(f"wait by b%16 (strip {w}):", " ".join(f"{np.median(wait[ph == k]):.0f}" for k in range(16)))
per = np.diff(t1[w, lo:hi + 1])
print(f"period by b%16 (strip {w}):", " ".join(f"{np.median(per[ph == k]):.0f}" for k in range(16)))
# the ratchet model: a strip's lag = the largest 5-block window of the strip above (+ detection)
for w in range(1, ns):
    if w % 4 == 0:
        continue
    d = np.diff(t1[w - 1, lo:hi + 1])
    win = np.convolve(d, np.ones(5, dtype=np.int64), "valid")
    lag = np.median(t1[w, lo:hi] - t1[w - 1, lo:hi])
    print(f"strip {w:2d}: lag {lag:6.0f}  5-window of strip {w-1}: mean {win.mean():6.0f} p99 {np.percentile(win, 99):6.0f} max {win.max():6.0f}")

# inter-workgroup hop, decomposed by column chunk (columns < 16c): strip 3 of ticket t publishes
# its block c+3 (elements < 16(c+4) = columns < 16c), the drain stores the granules, the loader of
# ticket t+1 feeds ring 0, strip 0 of ticket t+1 starts block c-1 (needs columns < 16c).
if hasattr(L, "gsa_dbg_kld"):
    d = np.zeros((8, 6400, 2), np.uint64)
    assert L.gsa_dbg_kld(d.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(d.nbytes)) == 0
    d = d.astype(np.int64)
    cs = np.arange(16, NB - 8)
    for t in range(min(7, ns // 4 - 1)):
        p3 = t2[4 * t + 3, cs + 3]
        dr = d[t, cs, 1]
        ld = d[t + 1, cs, 0]
        s0 = t1[4 * t + 4, cs - 1]
        ok = (dr > 0) & (ld > 0)
        print(f"ticket {t}->{t+1}: publish->drain med {np.median((dr - p3)[ok]):6.0f} | drain->loader med {np.median((ld - dr)[ok]):6.0f} "
              f"p90 {np.percentile((ld - dr)[ok], 90):6.0f} | loader->strip0 start med {np.median((s0 - ld)[ok]):6.0f} | total med {np.median((s0 - p3)[ok]):6.0f}")
    for t in range(min(8, ns // 4)):
        # intra-workgroup equivalent: strip w's start of block c-1 vs strip w-1's publish of block c+3
        w = 4 * t + 1
        print(f"ticket {t} intra (strip {w}): publish->start med {np.median(t1[w, cs - 1] - t2[w - 1, cs + 3]):6.0f}")
