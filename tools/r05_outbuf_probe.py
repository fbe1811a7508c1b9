"""The full batch's output buffer vs a fresh one: the 64-pair full batch (bench.py full_batch shape)
run three times in one process -- as bench.py runs it (after the headline), again, and again after
torch.cuda.empty_cache() -- each with pass times and the runtime fill kernel over the same
buffer (shard.gpu_batch_align timing: out_fill_*).  usage: r05_outbuf_probe.py [headline_first]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from gpuseqalign_amd import shard  # noqa: E402
from bench import subst_blosum62  # noqa: E402

pairs = shard.synthetic_batch(64, 18000, 22000, seed0=1000)
sub = subst_blosum62()
out_bytes = 4.0 * sum(len(y) * len(x) for y, x in pairs)
if "h" in sys.argv[1:]:
    # the headline first, in this process, as bench.py does
    from gpuseqalign_amd import formats as F
    x = F.synthetic_seq(100000, 100)
    import gpuseqalign_amd as gsa
    eng = gsa.Engine(0)
    y = F.mutate_seq(x, 101)
    for _ in range(3):
        eng.align_sparse(y, x, sub, -11, 256)
    eng.close()
pmc = "pmc" in sys.argv[1:]
runs = [("first", 0, False), ("second", 0, False), ("after empty_cache", 0, True)]
runs += [(f"shift {sh * 4 >> 10} KiB", sh, True) for sh in (16, 1 << 14, 1 << 18, 1 << 19, 3 << 18)]
if pmc:  # (under rocprofv3 --pmc: every state, one timed launch each, no misaligned base)
    runs = [r for r in runs if r[1] != 16]
pre = [a for a in sys.argv[1:] if a.startswith("pre")]
if pre:
    # a buffer of the batch's size allocated first and kept idle for N seconds, then freed into
    # torch's cache, so that the first run reuses memory the driver has had time to clear
    import time
    secs = float(pre[0][3:] or 10)
    tmp = torch.empty(int(out_bytes / 4) + (1 << 24), dtype=torch.int32, device="cuda:0")
    time.sleep(secs)
    print(f"(pre-allocated {tmp.numel() * 4 / 1e9:.1f} GB, idle {secs:.0f} s)", flush=True)
    del tmp
for label, sh, empty in runs:
    os.environ["GSA_PROBE_FLAT_SHIFT"] = str(sh)
    if empty:
        torch.cuda.empty_cache()
    tm = {}
    fn = shard.gpu_batch_align(device=0, mode="full", warmup=2, repeats=1 if pmc else 3,
                               out_budget_bytes=int(0.9 * 140e9), timing=tm)
    costs, secs = fn(list(range(64)), pairs, sub, -11)
    print(f"{label:18s} {secs * 1e3:8.3f} ms/launch  {out_bytes / secs / 1e12:5.2f} TB/s  pass1 {tm['pass1_ms']:.3f}  "
          f"pass2 {tm['pass2_ms']:.3f} ({out_bytes / tm['pass2_ms'] / 1e6:.0f} GB/s)  out_fill {tm['out_fill_ms']:.3f} ms "
          f"({tm['out_fill_bytes'] / tm['out_fill_ms'] / 1e6:.0f} GB/s)  clk {tm['clock_ghz_median']:.3f}  "
          f"base {tm['out_base']:#x} (mod 2 MiB {tm['out_base'] % (2 << 20):#x}, mod 1 GiB {tm['out_base'] % (1 << 30):#x})"
          + (f"  fresh fills {tm['fresh_fill0_ms']:.3f} / {tm['fresh_fill1_ms']:.3f} ms" if "fresh_fill0_ms" in tm else ""),
          flush=True)
