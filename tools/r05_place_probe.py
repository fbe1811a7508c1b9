"""Round-5 probe: does the full batch's pass-2 time depend on where its buffers land?  The 64-pair
full batch (the bench's full_batch workload, two launches, pitched) run N times in ONE process,
each after torch.cuda.empty_cache() and a spacer allocation of a different size placed before the
output buffer, so every run's matrices get other physical pages.  Prints pass times, the pass-2
clock, and the box's fill rate of a 16 GiB buffer at the same point.  JSON lines."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=6)
    ap.add_argument("--pairs", type=int, default=64)
    a = ap.parse_args()
    import torch
    import bench
    from gpuseqalign_amd import shard
    pairs = shard.synthetic_batch(a.pairs, 18000, 22000, seed0=1000)
    sub = bench.subst_blosum62()
    cells = sum((len(y) - 1) * (len(x) - 1) for y, x in pairs)
    nbytes = 4.0 * sum(len(y) * len(x) for y, x in pairs)
    for i in range(a.runs):
        torch.cuda.empty_cache()
        spacer = torch.empty(int((0.3 + 1.7 * i) * (1 << 28)), dtype=torch.int32, device="cuda:0")
        tm = {}
        costs, secs = shard.gpu_batch_align(0, mode="full", warmup=1, repeats=3, out_budget_bytes=int(0.9 * 140e9),
                                            timing=tm)(list(range(len(pairs))), pairs, sub, -11)
        box = bench.box_write_rate(0, gib=8, reps=3)
        del spacer
        print(json.dumps({"run": i, "spacer_GiB": round((0.3 + 1.7 * i) / 4, 3), "seconds": round(secs, 5),
                          "gcups": round(cells / secs / 1e9, 1), "TBps": round(nbytes / secs / 1e12, 3), **tm,
                          "box_GBps": box.get("GBps")}), flush=True)


if __name__ == "__main__":
    main()
