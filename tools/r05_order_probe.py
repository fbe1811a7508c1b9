"""Expansion task orders on one output buffer: the 64-pair full batch (bench.py full_batch shape)
with each GSA_EXPAND_RR order in turn on the same buffer (torch's cache hands the same block back),
then again on a second buffer (after torch.cuda.empty_cache()).  Pass-2 ms per order, 3 launches."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from gpuseqalign_amd import shard  # noqa: E402
from bench import subst_blosum62  # noqa: E402

pairs = shard.synthetic_batch(64, 18000, 22000, seed0=1000)
sub = subst_blosum62()
orders = sys.argv[1:] or ["1", "2", "4", "5", "6", "1"]
for buf in range(2):
    if buf:
        torch.cuda.empty_cache()
    line = []
    for o in orders:
        os.environ["GSA_EXPAND_RR"] = o
        tm = {}
        fn = shard.gpu_batch_align(device=0, mode="full", warmup=1, repeats=3, out_budget_bytes=int(0.9 * 140e9), timing=tm)
        fn(list(range(64)), pairs, sub, -11)
        line.append(f"rr{o} {tm['pass2_ms']:.2f}")
    print(f"buffer {buf} base {tm['out_base']:#x}: " + "  ".join(line), flush=True)
