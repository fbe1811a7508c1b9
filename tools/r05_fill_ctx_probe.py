"""What slows the runtime fill over the full batch's output buffer (4.6 TB/s inside
shard.gpu_batch_align vs 6.9 TB/s in a bare process): the same fill (torch fill_, int32, best of 3)
over a buffer of the batch's exact size, step by step as the context grows: bare; after creating
an Engine (gsa_ctx: two HIP streams, control words); after a torch side stream; after one full
batch on another buffer."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

N = 102216315136 // 4
dev = torch.device("cuda", 0)


def fill(label, buf, stream=None):
    best = None
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        if stream is None:
            e0.record(); buf.fill_(5); e1.record()
        else:
            e0.record(stream)
            with torch.cuda.stream(stream):
                buf.fill_(5)
            e1.record(stream)
        e1.synchronize()
        ms = e0.elapsed_time(e1)
        best = ms if best is None else min(best, ms)
    print(f"{label:44s} {best:8.3f} ms {N * 4 / (best * 1e-3) / 1e9:7.1f} GB/s", flush=True)


buf = torch.empty(N, dtype=torch.int32, device=dev)
fill("bare, exact size", buf)
import gpuseqalign_amd as gsa  # noqa: E402
eng = gsa.Engine(0)
fill("after Engine()", buf)
st = torch.cuda.Stream(device=dev)
fill("after a torch side stream (fill on it)", buf, st)
fill("after a torch side stream (fill on default)", buf)
del buf
torch.cuda.empty_cache()
buf = torch.empty(N, dtype=torch.int32, device=dev)
fill("new buffer, same context", buf)
small = [torch.empty(20000, dtype=torch.int32, device=dev) for _ in range(128)]
del buf
torch.cuda.empty_cache()
buf = torch.empty(N, dtype=torch.int32, device=dev)
fill("new buffer after 128 small tensors", buf)
eng.close()
