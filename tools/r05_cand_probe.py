"""Full-batch candidates on one output buffer after another: the 64-pair full batch (bench.py
full_batch shape) as one pair group (GSA_FULL_SPLIT=0) with expansion orders 1-6 and as two groups
(GSA_FULL_SPLIT=1) with orders 1 and 2, each fixed by GSA_EXPAND_RR, on the same buffer (torch's
cache hands the block back), then on NBUF-1 more buffers (torch.cuda.empty_cache() between).
Whole-launch ms (pass 1 + pass 2 event times) per candidate, 2 launches after 1 untimed."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from gpuseqalign_amd import shard  # noqa: E402
from bench import subst_blosum62  # noqa: E402

pairs = shard.synthetic_batch(64, 18000, 22000, seed0=1000)
sub = subst_blosum62()
cands = [("1", o) for o in ("1", "2", "4", "5", "6", "3")] + [("2", o) for o in ("1", "2", "4")]
nbuf = int(sys.argv[1]) if len(sys.argv) > 1 else 4
for buf in range(nbuf):
    if buf:
        torch.cuda.empty_cache()
    line = []
    for g, o in cands:
        os.environ["GSA_FULL_SPLIT"] = "0" if g == "1" else "1"
        os.environ["GSA_EXPAND_RR"] = o
        tm = {}
        fn = shard.gpu_batch_align(device=0, mode="full", warmup=1, repeats=2, out_budget_bytes=int(0.9 * 140e9), timing=tm)
        fn(list(range(64)), pairs, sub, -11)
        line.append(f"g{g}rr{o} {tm['pass1_ms'] + tm['pass2_ms']:.2f}")
    print(f"buffer {buf} base {tm['out_base']:#x}: " + "  ".join(line), flush=True)
