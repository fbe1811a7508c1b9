"""BASELINE configs[3]-style batch: many independent pairs sharded over the GPUs of one node
(gpuseqalign_amd/shard.py).  Single process = 1 GPU; under
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 tools/batch_bench.py
one rank per GPU over RCCL.  Prints one JSON line (rank 0): aggregate GCUPS over the timed
region (max over ranks), pairs, cells, concurrency.  --check verifies every align_cost
against the oracle (test infrastructure; small batches only)."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=64)
    ap.add_argument("--lo", type=int, default=18000)
    ap.add_argument("--hi", type=int, default=22000)
    ap.add_argument("--mode", default="sparse", choices=["sparse", "full"])
    ap.add_argument("--tileBx", type=int, default=512)
    ap.add_argument("--repeats", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--unpadded", action="store_true", help="full mode: adjcols pitch instead of gsa_full_pitch")
    a = ap.parse_args()

    import torch
    import torch.distributed as dist
    from gpuseqalign_amd import shard, formats as F

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    sd = F.read_subst_json(os.path.join(ROOT, "tests", "golden", "resrc", "subst.json"))
    subst = sd.matrix("blosum62") if rank == 0 else None
    pairs = shard.synthetic_batch(a.pairs, a.lo, a.hi, seed0=1000)
    fn = shard.gpu_batch_align(local, mode=a.mode, tileBx=a.tileBx, repeats=a.repeats, warmup=a.warmup,
                                pitched=not a.unpadded)
    rep = shard.shard_align(pairs, subst, -11, fn, device=torch.device("cuda", local) if world > 1 else None)
    if a.check and rank == 0:
        import oracle
        for r in rep.results:
            y, x = pairs[r.index]
            assert r.align_cost == oracle.fill_full(y, x, sd.matrix("blosum62"), -11)[1], r
    if rank == 0:
        print(json.dumps({"metric": "GCUPS, batch of independent NW-LG pairs (BASELINE configs[3] shape)",
                          "value": round(rep.gcups, 2), "unit": "GCUPS", "n_gpus": rep.world, "pairs": a.pairs,
                          "lengths": [a.lo, a.hi], "mode": a.mode, "pitched": a.mode == "full" and not a.unpadded, "tileBx": a.tileBx, "cells": rep.cells,
                          "seconds": round(rep.elapsed_s, 5), "repeats": a.repeats, "warmup": a.warmup,
                          "order": os.environ.get("GSA_BATCH_ORDER", "round-robin"),
                          "costs_head": [r.align_cost for r in rep.results[:4]], "checked": a.check}), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
