"""Plain-write rate of this box by buffer size: torch fill_ (the runtime's fill kernel) over int32
buffers of 4..96 GiB, best of 3 each, the buffer freed between sizes.  The full batch writes 102 GB
into one buffer; its pass 2 is compared with the fill over that same buffer in bench.py
(full_batch.passes.out_fill_*)."""
import torch

dev = torch.device("cuda", 0)
for gib in (4, 16, 32, 48, 64, 80, 96):
    buf = torch.empty(gib * (1 << 28), dtype=torch.int32, device=dev)
    buf.fill_(1)
    torch.cuda.synchronize(dev)
    best = None
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        buf.fill_(7)
        e1.record()
        e1.synchronize()
        ms = e0.elapsed_time(e1)
        best = ms if best is None else min(best, ms)
    # the same bytes as 16-GiB slices of the big buffer, one after the other
    sl = None
    if gib > 16:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 16 * (1 << 28)
        e0.record()
        for o in range(0, buf.numel(), n):
            buf[o:o + n].fill_(3)
        e1.record()
        e1.synchronize()
        sl = e0.elapsed_time(e1)
    print(f"{gib:3d} GiB  fill {best:8.3f} ms  {gib * (1 << 30) / (best * 1e-3) / 1e9:7.1f} GB/s"
          + (f"   as 16-GiB slices {sl:8.3f} ms {gib * (1 << 30) / (sl * 1e-3) / 1e9:7.1f} GB/s" if sl else ""),
          flush=True)
    del buf
    torch.cuda.empty_cache()
