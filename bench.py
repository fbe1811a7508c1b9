#!/usr/bin/env python3
"""bench.py -- NW-LG fill throughput (GCUPS) on MI355X, driver contract.

Workload (BASELINE.json configs[1]): one NW-LG 10k x 10k pair per rank and step, full int32
score matrix written to HBM (the plain/gpu3-6 representation), blosum62, gapo -11.  Inputs
(sequences, substitution table) are resident in HBM before the timed region; the output
matrix buffer is preallocated.  N>1: one process per GPU (torch.distributed, RCCL), pairs
shard across ranks with no data-path collective (weak scaling); RCCL only broadcasts the
substitution table and gathers per-pair align_costs.

Prints ONE JSON line (rank 0) with roofline (HBM-write bound, 4 B/cell) and cpu_baseline
(oracle restatement of cpu4-mt-diagrow, test infrastructure, timed on this host).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np

METRIC = "GCUPS (DP cell updates/s) + peak HBM GB/s, NW-LG N×M fill, 1/2/4/8 MI355X"
PEAK_HBM_GBPS = 8000.0  # MI355X_MICROARCH.md chip table (spec)


def load_pair(R, C):
    from gpuseqalign_amd import formats as F
    res = os.path.join(ROOT, "tests", "golden", "resrc")
    sd = F.read_subst_json(os.path.join(res, "subst.json"))
    if (R, C) == (10000, 10000):
        seqs = F.read_fasta(os.path.join(res, "seq_generated.fa"), sd.letter_map)
        Y, X = F.pair_arrays(F.parse_pair_line("len12124[:10000] len15390[:10000]", seqs), seqs)
        src = "reference resrc/seq_generated.fa: len12124[:10000] x len15390[:10000]"
    else:
        Y, X = F.synthetic_seq(R, 2), F.synthetic_seq(C, 3)
        src = "splitmix64 synthetic (seeds 2, 3)"
    return Y, X, sd.matrix("blosum62"), src


def full_kernel_name():
    """Name of the full-fill kernel libgsa launches (gsa_capi.hip: GSA_FULL_KERNEL, GSA_LANE_NS)."""
    if os.environ.get("GSA_FULL_KERNEL") == "strip":
        return "gsa::nw_strip_kernel<%s,0> (full)" % os.environ.get("GSA_FULL_NS", "1")
    ns = os.environ.get("GSA_LANE_NS", "4")   # nw_lane.h: kLaneNSDefault
    return "gsa::nw_lane_kernel<%s> (full, one row per lane)" % (ns if ns in ("1", "2", "3", "4") else "4")


def cpu_baseline(Y, X, sub, budget_s=8.0, threads=None):
    """cpu4-mt-diagrow restatement (oracle/, test infrastructure) on a bounded sample."""
    import oracle
    threads = threads or min(16, os.cpu_count() or 1)
    t_end = time.time() + budget_s
    reps, cells, t_tot = 0, 0, 0.0
    while time.time() < t_end or reps == 0:
        t0 = time.perf_counter()
        oracle.fill_full_mt(Y, X, sub, -11, blocksz=256, nthreads=threads)
        t_tot += time.perf_counter() - t0
        reps += 1
        cells += (len(Y) - 1) * (len(X) - 1)
    return {"value": round(cells / t_tot / 1e9, 4), "unit": "GCUPS", "cores": threads, "kind": "port",
            "sample": f"oracle cpu4-mt-diagrow restatement (blocksz 256, {threads} OpenMP threads), "
                      f"{reps} fills of the same {len(Y) - 1}x{len(X) - 1} pair, {t_tot:.1f} s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--R", type=int, default=10000)
    ap.add_argument("--C", type=int, default=10000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=8.0)
    a = ap.parse_args()

    import torch
    import torch.distributed as dist
    import gpuseqalign_amd as gsa

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    dev = torch.device("cuda", local if world > 1 else 0)

    Y, X, sub, src = load_pair(a.R, a.C)
    R, C = len(Y) - 1, len(X) - 1
    tY = torch.from_numpy(Y).to(dev)
    tX = torch.from_numpy(X).to(dev)
    tS = torch.from_numpy(sub).to(dev)
    if world > 1:
        dist.broadcast(tS, src=0)  # substitution table from rank 0 (RCCL over xGMI)
    score = torch.empty((R + 1) * (C + 1), dtype=torch.int32, device=dev)
    eng = gsa.Engine(dev.index)
    stream = torch.cuda.Stream(device=dev)
    sh = stream.cuda_stream

    def step():
        eng.fill_full_dev(tY.data_ptr(), R + 1, tX.data_ptr(), C + 1, tS.data_ptr(), 25, -11, score.data_ptr(), sh)

    with torch.cuda.stream(stream):
        for _ in range(a.warmup):
            step()
        eng.sync(sh)
        # per-launch kernel time (HIP events on the launch stream)
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for e0, e1 in evs:
            e0.record(stream)
            step()
            e1.record(stream)
        eng.sync(sh)
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([e0.elapsed_time(e1) for e0, e1 in evs]))
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        cost = score[-1:].clone()
        costs = [torch.zeros_like(cost) for _ in range(world)]
        dist.all_gather(costs, cost)
        costs = [int(c.item()) for c in costs]
    else:
        costs = [int(score[-1].item())]

    cells = float(R) * float(C)
    ms_per_step = elapsed * 1e3 / a.steps
    value = world * cells * a.steps / elapsed / 1e9
    bytes_per_launch = 4.0 * (R + 1) * (C + 1)
    achieved = bytes_per_launch / (kern_ms * 1e-3) / 1e9
    traffic = None
    tfile = os.path.join(ROOT, "profiles", "traffic.json")
    if os.path.exists(tfile):
        try:
            tj = json.load(open(tfile))
            if tj.get("R") == R and tj.get("C") == C and tj.get("kernel") == full_kernel_name():
                traffic = tj.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    if rank == 0:
        out = {
            "metric": METRIC, "value": round(value, 3), "unit": "GCUPS", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "int32", "data": f"synthetic ({src}); blosum62, gapo -11",
            "config": {"workload": f"NW-LG {R}x{C} full int32 score matrix in HBM (BASELINE configs[1])",
                       "R": R, "C": C, "pairs_per_rank": 1, "representation": "full (plain family)",
                       "parallelism": f"pair-sharded x{world}"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": PEAK_HBM_GBPS, "unit": "GB/s",
                         "frac": round(achieved / PEAK_HBM_GBPS, 4), "traffic": traffic,
                         "kernel": full_kernel_name(), "kernel_ms": round(kern_ms, 4),
                         "algorithmic_bytes_per_launch": bytes_per_launch},
            "align_costs": costs[:8],
        }
        if not a.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(Y, X, sub, budget_s=a.cpu_budget)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()
    eng.close()


if __name__ == "__main__":
    main()
