"""Probe for the config-4 share's last round: the time of 64 pairs whose
tickets make one round, on 8-strip (8, 4) tickets (2048 rows, 128 workgroups) and on 4-strip (4, 4)
tickets (1024 rows, 256 workgroups), beside two full rounds and the share itself.  usage:
r05_tail_probe.py  (GSA_KROW_NS set per case)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gpuseqalign_amd import shard, formats as F  # noqa: E402
from bench import subst_blosum62  # noqa: E402

sub = subst_blosum62()


def run(pairs, ns, label):
    if ns:
        os.environ["GSA_KROW_NS"] = str(ns)
    else:
        os.environ.pop("GSA_KROW_NS", None)
    fn = shard.gpu_batch_align(device=0, mode="sparse", tileBx=256, warmup=1, repeats=5)
    costs, secs = fn(list(range(len(pairs))), pairs, sub, -11)
    cells = sum((len(y) - 1) * (len(x) - 1) for y, x in pairs)
    print(f"{label:48s} ns={ns or 'auto'}  {secs * 1e3:8.3f} ms  {cells / secs / 1e12:6.2f} TCUPS", flush=True)
    return costs


def mk(n, R, C, seed):
    return [(F.synthetic_seq(R, seed + 2 * k), F.synthetic_seq(C, seed + 2 * k + 1)) for k in range(n)]


tail = mk(64, 4096, 20000, 7000)
c8 = run(tail, 8, "64 x (4096 x 20000): one round of (8,4)")
c4 = run(tail, 4, "64 x (4096 x 20000): one round of (4,4)")
assert c8 == c4
two = mk(64, 16384, 20000, 9000)
run(two, 8, "64 x (16384 x 20000): two rounds of (8,4)")
full = mk(64, 20480, 20000, 9000)
run(full, 8, "64 x (20480 x 20000): 2.5 rounds of (8,4)")
pairs = shard.synthetic_batch(512, 18000, 22000, seed0=1000)
w = [(len(y) - 1) * (len(x) - 1) for y, x in pairs]
parts = shard.lpt_partition(w, 8)
share = [pairs[i] for i in parts[0]]
run(share, 8, "config-4 LPT share 0 (64 pairs)")
run(share, 4, "config-4 LPT share 0 (64 pairs)")
