"""Row pitch of the full batch's matrices vs pass 2: gsa_full_pitch(adjcols) + 32 t ints (t = 0..7;
every pitch stays 1 mod 32, the layout the transposed stores assume), all on one allocation (sized
for the largest pitch, so torch's cache hands the same block back), then on a second allocation."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import gpuseqalign_amd as gsa  # noqa: E402
from gpuseqalign_amd import shard  # noqa: E402
from bench import subst_blosum62  # noqa: E402

pairs = shard.synthetic_batch(64, 18000, 22000, seed0=1000)
sub = subst_blosum62()
orig = gsa.full_pitch
pads = [int(a) for a in sys.argv[1:]] or list(range(8))
off = gsa.full_base_offset()


def need(t):
    return sum(-(-(off + len(y) * (orig(len(x)) + 32 * t)) // 32) * 32 for y, x in pairs)


top = need(max(pads))
for buf in range(2):
    if buf:
        torch.cuda.empty_cache()
    line = []
    for t in pads:
        gsa.full_pitch = lambda c, t=t: orig(c) + 32 * t
        os.environ["GSA_PROBE_FLAT_EXTRA"] = str(top - need(t))
        tm = {}
        fn = shard.gpu_batch_align(device=0, mode="full", warmup=2, repeats=3, out_budget_bytes=int(0.95 * 140e9),
                                   timing=tm)
        costs, _ = fn(list(range(64)), pairs, sub, -11)
        line.append(f"+{32 * t:3d}: {tm['pass2_ms']:.2f}")
    print(f"buffer {buf} base {tm['out_base']:#x}  pass2 ms by pitch pad (ints)  " + "  ".join(line), flush=True)
gsa.full_pitch = orig
