"""Diagnostic: the inter-workgroup link of the lane kernel, ticket 0 -> 1 (stamp build, GSA_LIB):
drain store times of ticket 0, poll issue/return times of ticket 1's loader.  Prints the poll
round trip, the time from a drain store to the first poll that returned its columns, and how
much of that is waiting for a poll to be issued.  s_memrealtime is 100 MHz: x24 = cycles at 2.4 GHz."""
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
n = 12000
buf = (ctypes.c_uint64 * n)()
assert L.gsa_debug_stamps(eng._h, buf, n) == 0
a = np.frombuffer(buf, dtype=np.uint64).astype(np.int64)
polls = a[4000:7000].reshape(-1, 3)
polls = polls[polls[:, 0] > 0]
drains = a[8000:12000].reshape(-1, 2)
drains = drains[drains[:, 0] > 0]
rtt = (polls[:, 1] - polls[:, 0]) * 24
print(f"polls {len(polls)}: round trip med {np.median(rtt):.0f} cyc, p10 {np.percentile(rtt, 10):.0f}, p90 {np.percentile(rtt, 90):.0f}")
gap = np.diff(polls[:, 0]) * 24
print(f"poll issue interval med {np.median(gap):.0f} cyc")
vis, wait_issue = [], []
for t, cols in drains:
    got = np.where(polls[:, 2] >= cols)[0]
    if len(got) == 0:
        continue
    k = got[0]
    vis.append((polls[k, 1] - t) * 24)
    after = np.where(polls[:, 0] >= t)[0]
    if len(after):
        wait_issue.append((polls[after[0], 0] - t) * 24)
vis, wait_issue = np.array(vis), np.array(wait_issue)
print(f"drain stores {len(drains)}: store -> returned by a poll med {np.median(vis):.0f} cyc (p10 {np.percentile(vis, 10):.0f}, p90 {np.percentile(vis, 90):.0f});"
      f" store -> next poll issue med {np.median(wait_issue):.0f}")
news = np.diff(np.concatenate([[0], polls[:, 2]]))
print(f"columns per poll: med {np.median(news):.0f}, polls with nothing new {np.mean(news <= 0) * 100:.0f} %")
