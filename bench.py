#!/usr/bin/env python3
"""bench.py -- NW-LG fill throughput (GCUPS) on MI355X, driver contract.

Headline workload (BASELINE.json north_star / configs[2]): ONE NW-LG
100k x 100k related pair per rank and step -- seqX = splitmix64 seed 100, seqY = seqX with 15 %
substitutions + 2 % indels (seed 101) -- filled into the sparse tile-header (mlsp) form
(tileHrowMat / tileHcolMat, tileBx 256), blosum62, gapo -11.  The path replaced is
NwAlign_Gpu9_Mlsp_DiagDiagDiag (nwalign_gpu9_mlsp_diagdiagdiag.cu:368-722) timed as align.calc
(benchmark.cpp:473).  Inputs (sequences, substitution table) are resident in HBM before the
timed region; the header buffers are preallocated.  The fill's align_cost is checked against
the oracle golden tests/golden/config3_100k.json (data; no oracle code runs here).

N>1: one process per GPU (torch.distributed, RCCL); every rank fills its own config-3 pair
(weak scaling, no data-path collective: RCCL only broadcasts the substitution table and
gathers align_costs / max-reduces the time).  The `config4` field is BASELINE configs[3]: the
512 pairs of 18-22k (shard.synthetic_batch, seeds 1000+k) LPT-sharded over the N ranks
(strong scaling: fixed total work), each rank's share in one persistent batched launch, every
align_cost checked against tests/golden/config4_pairs.json.  `fill_10k_full` is configs[1].

Roofline: the sparse fill does not stream HBM (headers are ~0.07 B/cell); it is bound by int32
VALU issue.  Algorithmic work = 5 int ops per cell (3 add + 2 max, UpdateScore,
nwalign_cpu1_st_row.cpp:4-10); peak = 256 CU x 4 SIMD x 32 lanes x 2.4 GHz = 78.6 T lane-ops/s
(MI355X_MICROARCH.md: SIMD-32, wave64 VALU over 2 cycles).  cpu_baseline: the oracle's
cpu4-mt-diagrow restatement (test infrastructure) on a bounded 20k x 20k prefix of the same pair.
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
PEAK_HBM_GBPS = 8000.0                       # MI355X_MICROARCH.md chip table (spec)
PEAK_VALU_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12  # int32 lane-ops/s, 78.6 T
OPS_PER_CELL = 5
TILE_BX = 256


def subst_blosum62():
    from gpuseqalign_amd import formats as F
    return F.read_subst_json(os.path.join(ROOT, "tests", "golden", "resrc", "subst.json")).matrix("blosum62")


def config3_pair():
    from gpuseqalign_amd import formats as F
    X = F.synthetic_seq(100000, 100)
    return F.mutate_seq(X, 101), X


def config2_pair():
    from gpuseqalign_amd import formats as F
    res = os.path.join(ROOT, "tests", "golden", "resrc")
    sd = F.read_subst_json(os.path.join(res, "subst.json"))
    seqs = F.read_fasta(os.path.join(res, "seq_generated.fa"), sd.letter_map)
    return F.pair_arrays(F.parse_pair_line("len12124[:10000] len15390[:10000]", seqs), seqs)


def load_golden(name):
    p = os.path.join(ROOT, "tests", "golden", name)
    if not os.path.exists(p):
        return None
    with open(p) as f:
        return json.load(f)


def lane_ns():
    """Lane strips per workgroup of full fills, as gsa_capi.hip's lane_ns() reads GSA_LANE_NS."""
    v = os.environ.get("GSA_LANE_NS", "")
    return int(v) if v in ("1", "2", "3", "4", "6", "8") else 4


def full_kernel_name(single):
    """Kernels of a full fill (gsa_capi.hip full_twopass): the two-pass fill (pass 1: K-rows XR
    instance, (4, 4) for one pair and (8, 4) for a batch that overfills the chip; pass 2: the
    streamed tile expansion, 7 tile waves + a loader wave per workgroup), fused into one launch for a
    single pair; or under GSA_FULL_KERNEL=lane the one-pass lane fill."""
    if os.environ.get("GSA_FULL_KERNEL", "") == "lane":
        return lane_kernel_name(single)
    fm = os.environ.get("GSA_FULL_FUSED", "1")
    if single and fm != "0":
        return ("gsa::nw_full_fused_kernel<4,8,true,3> for R x C > 2^30 (pass-1 strips stage row 64m in LDS for a "
                "storer wave), <4,8,true,4> below (strips store row 64m themselves) (both passes in one launch: (4, 4) "
                "K-rows pass-1 tickets "
                "publishing per-strip progress, then the streamed expansion: a loader wave per workgroup stages "
                "each 448-row x 512-column task once pass 1 has passed it, 7 tile waves store parallelogram tiles)")
    ns = 4 if single else 8
    name = (f"gsa::nw_krow_kernel<{ns},4,1024,2,true> (pass 1: sparse wavefront keeping every 64th row and the "
            f"256-column header columns) + gsa::nw_expand_stream_kernel (pass 2: every 64 x 512 tile recomputed, "
            f"7 tile waves + a loader wave per workgroup)")
    if not single and os.environ.get("GSA_FULL_SPLIT", "") != "0":
        name += ("; a batch whose pass-1 tickets end in a short round may run as two pair groups (tuned on its "
                 "first launches, pipelined_groups in passes): group A (the full rounds) on the caller's stream, "
                 "group B's pass 1 on a high-priority stream after A's, beside A's expansion")
    return name


def lane_kernel_name(single):
    """The lane instantiation a full fill runs (nw_lane.hip launch_lane_fill): <NS, feeder wave,
    paired stores>; the feeder wave for single pairs at NS = 4 (GSA_LANE_FEED), paired stores for
    batches (GSA_LANE_PAIR)."""
    ns = lane_ns()
    fe, pe = os.environ.get("GSA_LANE_FEED", ""), os.environ.get("GSA_LANE_PAIR", "")
    fd = ns == 4 and (int(fe) != 0 if fe else single)
    pair = (int(pe) != 0 if pe else not fd) if ns == 4 else True
    return f"gsa::nw_lane_kernel<{ns},{'true' if fd else 'false'},{'true' if pair else 'false'}>"


def sparse_kernel_name():
    """The K-rows instantiation a single-pair sparse fill runs (gsa_capi.hip: GSA_KROW_NS / GSA_KROW_K,
    default (4, 4); the profile ring is 512 columns with 2 strips, 1024 otherwise; GSA_KROW_Q8=0: the
    int16 profile instance instead of the int8 one)."""
    ns, k = os.environ.get("GSA_KROW_NS", "4"), os.environ.get("GSA_KROW_K", "4")
    ok = (k in ("2", "4") and ns in ("2", "4")) or (k == "4" and ns == "8")
    ns, k = (int(ns), int(k)) if ok else (4, 4)
    lw = 512 if ns == 2 else 1024
    q8 = os.environ.get("GSA_KROW_Q8", "1") != "0"
    return (f"gsa::nw_krow_kernel<{ns},{k},{lw},false,{'true' if q8 else 'false'}> (sparse, K = {k} rows per lane, "
            f"{'int8' if q8 else 'int16'} column profile" + ("; the int16 instance behind it is a ~5 us no-op)" if q8 else ")"))


def cpu_topology():
    """(usable logical CPUs, physical cores among them, cgroup CPU quota or None, nproc)."""
    try:
        cpus = sorted(os.sched_getaffinity(0))
    except AttributeError:
        cpus = list(range(os.cpu_count() or 1))
    phys = set()
    try:
        with open("/proc/cpuinfo") as f:
            for line in f.read().split("\n\n"):
                d = dict(kv.split(":", 1) for kv in line.split("\n") if ":" in kv)
                d = {k.strip(): v.strip() for k, v in d.items()}
                if "processor" in d and int(d["processor"]) in cpus:
                    phys.add((d.get("physical id", "0"), d.get("core id", d["processor"])))
    except Exception:
        phys = set()
    quota = None
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(p)
    except Exception:
        pass
    return len(cpus), (len(phys) or len(cpus)), quota, os.cpu_count()


def cpu_baseline(Y, X, sub, budget_s=20.0, n=20000):
    """cpu4-mt-diagrow restatement (oracle/, test infrastructure) on a bounded n x n prefix of the
    headline pair, timed at the physical core count and at the process's CPU share."""
    import oracle
    ncpu, phys, quota, nproc = cpu_topology()
    share = max(1, min(phys, int(quota) if quota else phys))
    Yp, Xp = Y[:n + 1], X[:n + 1]
    cands = sorted({phys, share, min(16, phys)}, reverse=True)
    runs = {}
    for th in cands:
        t_end = time.time() + budget_s / len(cands)
        reps, t_tot = 0, 0.0
        while time.time() < t_end or reps == 0:
            t0 = time.perf_counter()
            oracle.fill_full_mt(Yp, Xp, sub, -11, blocksz=256, nthreads=th)
            t_tot += time.perf_counter() - t0
            reps += 1
        runs[th] = (n * n * reps / t_tot / 1e9, reps, t_tot)
    best = max(runs, key=lambda t: runs[t][0])
    v, reps, t_tot = runs[best]
    return {"value": round(v, 4), "unit": "GCUPS", "cores": best, "kind": "port",
            "sample": (f"oracle cpu4-mt-diagrow restatement (blocksz 256, OpenMP), {reps} fills of the "
                       f"{n}x{n} prefix of the config-3 pair in {t_tot:.1f} s at {best} threads; host: nproc "
                       f"{nproc}, {ncpu} CPUs in the affinity mask, {phys} physical cores, cgroup quota "
                       f"{quota if quota else 'none'}; threads tried: "
                       + ", ".join(f"{t}: {runs[t][0]:.3f} GCUPS" for t in sorted(runs)))}


# GSA_BENCH_REHEARSE=1 (test only): N ranks share cuda:0 and talk over gloo with CPU tensors, to
# exercise the N > 1 code path on a one-GPU box; its numbers mean nothing (the GPU is shared)
REHEARSE = os.environ.get("GSA_BENCH_REHEARSE") == "1"


def gpu_fields(world):
    """n_gpus / parallelism / rehearsal of the JSON line: a rehearsal's ranks share cuda:0, so it
    reports the devices it used (1) and says what it was, never a multi-GPU result."""
    if REHEARSE:
        return {"n_gpus": 1, "rehearsal": True,
                "parallelism": f"REHEARSAL: {world} gloo ranks sharing one GPU (not a scaling result)"}
    return {"n_gpus": world, "rehearsal": False, "parallelism": f"pair-sharded x{world}"}


def coll_dev(dev):
    """Where collective tensors live: the rank's GPU (RCCL), or the CPU in a gloo rehearsal."""
    import torch
    return torch.device("cpu") if REHEARSE else dev


def timed_steps(step, stream, dev, steps, warmup, world, eng):
    import torch
    import torch.distributed as dist
    with torch.cuda.stream(stream):
        for _ in range(warmup):
            step()
        eng.sync(stream.cuda_stream)
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for e0, e1 in evs:
            e0.record(stream)
            step()
            e1.record(stream)
        eng.sync(stream.cuda_stream)
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([e0.elapsed_time(e1) for e0, e1 in evs]))
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=coll_dev(dev))
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed, kern_ms


def traffic_for(name, R, C, kernel):
    p = os.path.join(ROOT, "profiles", name)
    if not os.path.exists(p):
        return None
    try:
        tj = json.load(open(p))
        if tj.get("R") == R and tj.get("C") == C and tj.get("kernel") == kernel:
            return tj.get("hbm_bytes_per_launch")
    except Exception:
        return None
    return None


def bench_config4(world, rank, local, n_pairs):
    """BASELINE configs[3]: n_pairs pairs of 18-22k, LPT-sharded over the ranks (strong scaling)."""
    from gpuseqalign_amd import shard
    pairs = shard.synthetic_batch(n_pairs, 18000, 22000, seed0=1000)
    sub = subst_blosum62()
    rep = shard.shard_align(pairs, sub, -11, shard.gpu_batch_align(device=local, mode="sparse", tileBx=TILE_BX,
                                                                warmup=1, repeats=3),
                            device=f"cuda:{local}" if world > 1 and not REHEARSE else None)
    gold = load_golden("config4_pairs.json")
    costs = [r.align_cost for r in rep.results]
    match = None
    if gold is not None and gold.get("n_pairs", 0) >= n_pairs:
        match = sum(int(a == b) for a, b in zip(costs, gold["align_cost"][:n_pairs]))
    return {"workload": f"BASELINE configs[3]: {n_pairs} NW-LG pairs, lengths uniform in [18000, 22000] "
                        f"(seeds 1000+k), sparse tile headers (tileBx {TILE_BX}), LPT-sharded over {world} rank(s), "
                        "one persistent batched launch per rank (1 untimed + 3 timed launches; seconds per launch)",
            "value": round(rep.gcups, 2), "unit": "GCUPS", "scaling": "strong", "cells": rep.cells,
            "seconds": round(rep.elapsed_s, 4), "pairs": n_pairs,
            "pairs_matching_golden": match, "golden_pairs": None if gold is None else gold.get("n_pairs")}


def bench_config4_rank_share(local, n_pairs, cfg4, ranks=8):
    """One-GPU fact that bounds the 8-GPU strong scaling of configs[3]: every rank's LPT share
    (shard.lpt_partition(weights, 8)[k], ~64 pairs) timed as the one launch that rank would run,
    one share after the other on this GPU.  An 8-GPU run cannot beat the slowest share, so
    projected_8gpu_speedup = (time of all n_pairs on one GPU) / (slowest share); the longest pair
    of share 0 alone is the critical path under it."""
    from gpuseqalign_amd import shard
    pairs = shard.synthetic_batch(n_pairs, 18000, 22000, seed0=1000)
    sub = subst_blosum62()
    weights = [(len(y) - 1) * (len(x) - 1) for y, x in pairs]
    parts = shard.lpt_partition(weights, ranks)
    gold = load_golden("config4_pairs.json")
    fn = shard.gpu_batch_align(device=local, mode="sparse", tileBx=TILE_BX, warmup=1, repeats=3)
    shares, match = [], 0
    for idx in parts:
        costs, secs = fn(idx, pairs, sub, -11)
        if gold is not None:
            match += sum(int(c == gold["align_cost"][i]) for i, c in zip(idx, costs))
        cells = sum(weights[i] for i in idx)
        shares.append({"pairs": len(idx), "cells": cells, "seconds": round(secs, 6),
                       "gcups": round(cells / secs / 1e9, 2)})
    longest = max(parts[0], key=lambda i: weights[i])
    _, t1 = shard.gpu_batch_align(device=local, mode="sparse", tileBx=TILE_BX, warmup=1, repeats=3)(
        [longest], pairs, sub, -11)
    slowest = max(sh["seconds"] for sh in shares)
    t_all = cfg4["seconds"] if cfg4 else None
    return {"workload": f"configs[3] LPT shares for {ranks} ranks, each timed alone on this GPU (one launch per "
                        "share, 1 untimed + 3 timed launches)",
            "ranks": ranks, "share0": shares[0], "shares_seconds": [sh["seconds"] for sh in shares],
            "slowest_share_seconds": slowest,
            "share_gcups": round(sum(weights) / ranks / slowest / 1e9, 2),
            "projected_8gpu_gcups": round(sum(weights) / slowest / 1e9, 2),
            "projected_8gpu_speedup": None if t_all is None else round(t_all / slowest, 3),
            "single_pair": {"pair": int(longest), "R": len(pairs[longest][0]) - 1, "C": len(pairs[longest][1]) - 1,
                            "seconds": round(t1, 6)},
            "pairs_matching_golden": match if gold is not None else None}


CLOCK_GHZ = 2.4          # MI355X_MICROARCH.md chip table (max clock)
VALU_ISSUE_CYC = 4       # one wave alone issues one VALU per 4 cycles (MI355X_MICROARCH.md constants table)


def critical_path(C, nStrips, valu_per_step, kern_ms, rows_per_strip):
    """Design bound of one pair's wavefront fill: the last strip cannot finish before C steps
    after it starts, and it starts nStrips x 64 steps after the first (each strip trails the one
    above by at least the 64-lane skew); a step is at least its VALU at one wave's issue rate."""
    step_cyc = valu_per_step * VALU_ISSUE_CYC
    steps = C + nStrips * 64
    bound_ms = steps * step_cyc / (CLOCK_GHZ * 1e9) * 1e3
    return {"model": f"(C + strips x 64) steps x {valu_per_step} VALU x {VALU_ISSUE_CYC} cycles / {CLOCK_GHZ} GHz",
            "strips": nStrips, "rows_per_strip": rows_per_strip, "steps": steps, "step_cycles_bound": step_cyc,
            "bound_ms": round(bound_ms, 4), "frac": round(bound_ms / kern_ms, 4),
            "step_cycles_achieved": round(kern_ms * 1e-3 * CLOCK_GHZ * 1e9 / steps, 1)}


def bench_full_batch(world, rank, local, n_pairs):
    """Full-matrix family at throughput (the plain gpu3-gpu6 slots, nwalign_gpu3_ml_diagdiag.cu:
    288-596): n_pairs of the configs[3] pairs (18-22k, seeds 1000+k) as full int32 matrices in ONE
    persistent launch; the bound is HBM writes (4 B per cell).  Every align_cost (the last cell)
    is checked against the oracle goldens of tests/golden/config4_pairs.json."""
    from gpuseqalign_amd import shard
    pairs = shard.synthetic_batch(n_pairs, 18000, 22000, seed0=1000)
    sub = subst_blosum62()
    tm = {}
    # 6 untimed launches: the library runs a batch's first launch untimed, times its four candidates
    # (one or two pair groups x two expansion task orders) on the next four and keeps the fastest
    # (gsa_capi.hip enqueue_full); the first launch's time is reported as first_launch_ms
    rep = shard.shard_align(pairs, sub, -11, shard.gpu_batch_align(device=local, mode="full", warmup=6, repeats=3,
                                                                out_budget_bytes=int(0.9 * 140e9), timing=tm),
                            device=f"cuda:{local}" if world > 1 and not REHEARSE else None)
    gold = load_golden("config4_pairs.json")
    costs = [r.align_cost for r in rep.results]
    match = None if gold is None else sum(int(a == b) for a, b in zip(costs, gold["align_cost"][:n_pairs]))
    out_bytes = 4.0 * sum(len(y) * len(x) for y, x in pairs)
    gbps = out_bytes / rep.elapsed_s / 1e9
    box = box_write_rate(local)
    return {"workload": f"{n_pairs} NW-LG pairs of BASELINE configs[3] (18-22k, seeds 1000+k) as FULL int32 score "
                        f"matrices ({out_bytes / 1e9:.1f} GB), one persistent launch, LPT-sharded over {world} rank(s) "
                        "(6 untimed + 3 timed launches; seconds per launch)",
            "value": round(rep.gcups, 2), "unit": "GCUPS", "scaling": "strong", "seconds": round(rep.elapsed_s, 4),
            "kernel": full_kernel_name(False),
            "layout": "pitched: row pitch gsa_full_pitch(adjcols) = 1 mod 32, cell (1,0) on a 128-byte boundary",
            "hbm_write_GBps": round(gbps * world, 1), "hbm_frac": round(gbps / PEAK_HBM_GBPS, 4),
            "bound": "hbm (4 B written per cell; MI355X 8 TB/s spec)",
            "pmc_write_over_algorithmic": pmc_write_ratio(n_pairs, full_kernel_name(False)),
            "passes": pass_fields(tm, out_bytes / world),
            "first_launch_ms": None if "first_launch_ms" not in tm else round(tm["first_launch_ms"], 4),
            "first_launch_wall_ms": None if "first_launch_wall_ms" not in tm else round(tm["first_launch_wall_ms"], 4),
            "box_fill": box,
            "over_box_fill": round(gbps / box["GBps"], 4) if box and "GBps" in box else None,
            "pairs": n_pairs, "pairs_matching_golden": match}


def bench_full100k(dev, eng, tS, sh, stream, steps, warmup, world):
    """The north star's own pair as a FULL matrix: the config-3 100k x 100k NW-LG related pair (9.99e9
    cells, 40 GB int32) in HBM, pitched layout (gsa_fill_full_pitched_dev: row pitch gsa_full_pitch,
    cell (1, 0) on a 128-byte boundary), the fused two-pass fill in one launch.  Bound: HBM writes,
    4 B per cell.  align_cost (the last cell) against the oracle golden; the device hash / trace /
    recurrence check of the same matrix are tests/test_gpu_full100k.py's."""
    import torch
    import gpuseqalign_amd as gsa
    Y, X = config3_pair()
    R1, C1 = len(Y), len(X)
    ld, off = gsa.full_pitch(C1), gsa.full_base_offset()
    try:
        buf = torch.empty((R1 - 1) * ld + C1 + off + 64, dtype=torch.int32, device=dev)
    except RuntimeError as ex:  # (no room: the field says so)
        return {"error": str(ex)[:120]}
    tY, tX = torch.from_numpy(Y).to(dev), torch.from_numpy(X).to(dev)
    base = buf.data_ptr() + 4 * off

    def step():
        eng.fill_full_dev(tY.data_ptr(), R1, tX.data_ptr(), C1, tS.data_ptr(), 25, -11, base, sh, ld=ld)

    el, km = timed_steps(step, stream, dev, steps, warmup, world, eng)
    cost = int(buf[off + (R1 - 1) * ld + C1 - 1].item())
    gold = load_golden("config3_100k.json")
    b = 4.0 * R1 * C1
    del buf
    torch.cuda.empty_cache()
    return {"workload": "BASELINE configs[2] pair (100k x 100k NW-LG, related) as a FULL int32 score matrix "
                        f"({b / 1e9:.1f} GB) in HBM, pitched rows (ld {ld}), one fused launch per step",
            "value": round(world * (R1 - 1) * (C1 - 1) * steps / el / 1e9, 1), "unit": "GCUPS",
            "ms_per_step": round(el * 1e3 / steps, 4), "kernel_ms": round(km, 4), "steps": steps,
            "kernel": full_kernel_name(True),
            "hbm_write_GBps": round(b / (km * 1e-3) / 1e9, 1),
            "hbm_frac": round(b / (km * 1e-3) / 1e9 / PEAK_HBM_GBPS, 4),
            "bound": "hbm (4 B written per cell; MI355X 8 TB/s spec)",
            "pmc_write_over_algorithmic": pmc_full100k_ratio(),
            "rocprof": "profiles/r06_full100k_kernel_stats.csv (nw_full_fused_kernel<4, 8, true, 3>, this fill alone)",
            "align_cost": cost,
            "golden_align_cost": None if gold is None else gold["pairs"]["related"]["align_cost"]}


def pmc_full100k_ratio():
    """WRITE_SIZE of the fused 100k x 100k fill over its matrix bytes (profiles/r06_pmc.json)."""
    try:
        return json.load(open(os.path.join(ROOT, "profiles", "r06_pmc.json")))["pmc"]["f"]["write_over_algorithmic"]
    except Exception:
        return None


def box_write_rate(local, gib=16, reps=5):
    """What this box's HBM takes in plain writes: torch fill_ of a 16 GiB int32 buffer (the runtime's
    fill kernel, 16-byte stores, every CU), best of 5.  The full batch's rate over this one separates
    the kernel from the box: the same build's pass 2 ran 18.8 ms on one box and 25.3 on another at a
    higher shader clock (profiles/r05_pipe_ab.txt)."""
    import torch
    try:
        dev = torch.device("cuda", local)
        buf = torch.empty(gib * (1 << 28), dtype=torch.int32, device=dev)
        buf.fill_(1)
        torch.cuda.synchronize(dev)
        best = None
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            buf.fill_(7)
            e1.record()
            e1.synchronize()
            ms = e0.elapsed_time(e1)
            best = ms if best is None else min(best, ms)
        del buf
        torch.cuda.empty_cache()
        return {"what": f"torch fill_ of {gib} GiB int32, best of {reps}", "ms": round(best, 4),
                "GBps": round(gib * (1 << 30) / (best * 1e-3) / 1e9, 1)}
    except Exception as ex:  # (no room: the field is left out)
        return {"error": str(ex)[:120]}


def pass_fields(tm, rank_bytes):
    """This rank's last timed launch, pass by pass (HIP events on the launch stream,
    gsa_last_full_timing), and pass 2's effective shader clock (per-workgroup s_memtime /
    s_memrealtime): pass 2 alone is HBM-write bound, and its rate follows the clock the box runs."""
    if not tm:
        return None
    out = dict(tm)
    p1, p2 = tm.get("pass1_ms"), tm.get("pass2_ms")
    if p2:
        out["pass2_write_GBps"] = round(rank_bytes / (p2 * 1e-3) / 1e9, 1)
        out["pass2_hbm_frac"] = round(rank_bytes / (p2 * 1e-3) / 1e9 / PEAK_HBM_GBPS, 4)
    if p1 is not None and p2:
        out["pass1_share"] = round(p1 / (p1 + p2), 4)
    # the runtime's fill kernel over the same output buffer: a box whose pages slow every writer
    # shows it here, one whose pass 2 alone is slow does not
    fm, fb = tm.get("out_fill_ms"), tm.get("out_fill_bytes")
    if fm and fb:
        out["out_fill_ms"] = round(fm, 4)
        out["out_fill_GBps"] = round(fb / (fm * 1e-3) / 1e9, 1)
        if p2:
            out["pass2_over_out_fill"] = round(fm / p2 * rank_bytes / fb, 4)
    if tm.get("pipelined_groups") == 2:
        out["groups_note"] = ("two pair groups: pass1_ms is group A's pass 1 alone; pass2_ms everything after "
                              "(A's expansion beside B's pass 1, then B's expansion), so pass2 rates are lower bounds")
    out["nominal_clock_ghz"] = CLOCK_GHZ
    return out


def pmc_write_ratio(n_pairs, kernel):
    """HBM bytes written (PMC WRITE_SIZE of both passes, profiles/r06_pmc_full_batch.json, collected
    by tools/r06_prof.sh on the same batch) over the matrix bytes, or None for another
    shape/kernel: the physical write rate is hbm_write_GBps times this."""
    p = os.path.join(ROOT, "profiles", "r06_pmc_full_batch.json")
    try:
        j = json.load(open(p))
        if n_pairs == 64 and j.get("kernel", "").split(" ")[0] == kernel.split(" ")[0]:
            return round(j["write_over_algorithmic"], 4)
    except Exception:
        return None
    return None


CFG5 = [("SW-LG", -11, -11, True), ("NW-AG", -11, -1, False)]


def score_kernel_name(go, ge, local, substsz=25, R=50000, C=50000):
    """The kernel gsa_score_dev runs (gsa_capi.hip score_dev_impl): the K-rows score kernel unless
    GSA_SCORE_KERNEL=strip, SW with ge > 0, or its LDS does not fit (a 25-letter table fits); the
    strip kernel's score modes otherwise (4 strips per workgroup).  NW on R rows, R a multiple of K
    and each half >= 4 tickets (or the same of C, transposed): from both ends (score_bidi: two
    halves in one launch, K = 2)."""
    mode = (5 if go == ge else 4) if local else (6 if go == ge else 3)
    mname = (("kModeScoreSWL" if go == ge else "kModeScoreSW") if local else
             ("kModeScoreAGL" if go == ge else "kModeScoreAG"))
    krow = os.environ.get("GSA_SCORE_KERNEL", "") != "strip" and (not local or ge <= 0) and substsz <= 32
    # rows per lane: 4 for NW-LG, 2 otherwise (GSA_SCORE_K forces one); the int8-profile instance at
    # 4 rows per lane (gsa_capi.hip score_ag_strip; GSA_KROW_Q8 0 / 2: never / always)
    kenv = os.environ.get("GSA_SCORE_K", "")
    k = int(kenv) if kenv in ("2", "4") else (4 if (not local and go == ge) else 2)
    bidi_env = os.environ.get("GSA_SCORE_BIDI", "1")
    kb = int(kenv) if kenv in ("2", "4") else 2
    splits = lambda rows: rows % kb == 0 and rows >= 2 * kb and (bidi_env == "2" or rows >= 8 * 64 * kb * 4)
    bidi = krow and not local and bidi_env != "0" and (splits(R) or splits(C))
    # SW: by rows only, three pairs (top forward, bottom reversed, bottom forward from a fresh
    # border), back to one direction when an alignment through the split decides the result
    bidi_sw = (krow and local and bidi_env != "0" and os.environ.get("GSA_SCORE_BIDI_SW", "1") != "0"
               and splits(R))
    if bidi or bidi_sw:
        k = kb
    q8env = os.environ.get("GSA_KROW_Q8", "1")
    q8 = q8env != "0" and (q8env == "2" or k == 4)
    tag = (", both ends: two halves in one launch" if bidi else
           ", both ends: top forward, bottom reversed and bottom fresh in one launch" if bidi_sw else "")
    return (f"gsa::nw_kscore_kernel<{mode}, {'true' if q8 else 'false'}, {k}> ({mname}{tag})" if krow else
            f"gsa::nw_strip_kernel<4,{mode}> ({mname}, strip kernel)")


def bench_config5(dev, eng, steps, warmup, cpu_sample, rank, world):
    """BASELINE configs[4]: score-only SW-LG and NW-AG (gapo -11, gape -1) on the 50k x 50k random
    pair (seeds 200/201), inputs resident in HBM; kernel time from HIP events around each launch
    (gsa_score_dev is synchronous).  Scores and end cells checked against the oracle goldens
    (tests/golden/config5_50k.json, oracle/score_oracle.c).  cpu_baseline: the oracle's tiled
    OpenMP score wavefront (cpu4-mt-diagrow shape) on a bounded prefix sample, rank 0 at N = 1."""
    import torch
    from gpuseqalign_amd import formats as F
    Y, X = F.synthetic_seq(50000, 200), F.synthetic_seq(50000, 201)
    sub = subst_blosum62()
    y, x, s = (torch.from_numpy(np.ascontiguousarray(a, dtype=np.int32)).to(dev) for a in (Y, X, sub))
    gold = load_golden("config5_50k.json")
    R, C = len(Y) - 1, len(X) - 1
    out = {}
    for name, go, ge, local in CFG5:
        run = lambda: eng.score_dev(y.data_ptr(), len(Y), x.data_ptr(), len(X), s.data_ptr(), 25, go, ge, local)
        for _ in range(warmup):
            run()
        ks = []
        t0 = time.perf_counter()
        for _ in range(steps):
            r = run()
            ks.append(r["kernel_ms"])
        wall = (time.perf_counter() - t0) / steps
        g = None if gold is None else gold["modes"][name]
        ok = None if g is None else (r["score"], r["i_end"], r["j_end"]) == (g["score"], g["i_end"], g["j_end"])
        kms = float(np.mean(ks))
        out[name] = {"value": round(R * C / kms / 1e6, 2), "unit": "GCUPS", "kernel_ms": round(kms, 4),
                     "ms_per_call": round(wall * 1e3, 4), "score": r["score"], "end": [r["i_end"], r["j_end"]],
                     "golden_match": ok, "gapo": go, "gape": ge, "local": local,
                     "kernel": score_kernel_name(go, ge, local, R=R, C=C)}
        if cpu_sample > 0 and rank == 0 and world == 1:
            import oracle
            ncpu, phys, quota, nproc = cpu_topology()
            th = max(1, min(phys, int(quota) if quota else phys))
            m = cpu_sample
            t1 = time.perf_counter()
            oracle.score_ag(Y[:m + 1], X[:m + 1], sub, go, ge, local, mt=True, blocksz=256, nthreads=th)
            cs = time.perf_counter() - t1
            out[name]["cpu_baseline"] = {"value": round(m * m / cs / 1e9, 3), "unit": "GCUPS", "cores": th,
                                         "kind": "port",
                                         "sample": f"oracle score_oracle.c tiled OpenMP wavefront (blocksz 256) on the "
                                                   f"{m}x{m} prefix of the same pair, {cs:.1f} s at {th} threads"}
    return {"workload": "BASELINE configs[4]: score-only 50000x50000 random pair (synthetic seeds 200/201), blosum62",
            "modes": out}


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launch_ranks(gpus):
    """--gpus N and the process layout, settled before any GPU call.  Under a launcher (WORLD_SIZE
    set) the launcher's world must equal --gpus, else exit 2: a line must never say N GPUs for a
    different number of ranks.  Without one, --gpus N > 1 starts N ranks itself, one process per
    GPU, through torch.distributed.run on 127.0.0.1 (a child process: this one never initialises
    the GPU), and returns the child's exit code.  None: go on as this rank."""
    if gpus < 1:
        print(f"bench.py: --gpus {gpus} < 1", file=sys.stderr)
        return 2
    ws = os.environ.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != gpus:
            print(f"bench.py: --gpus {gpus} but WORLD_SIZE={ws}: the launcher started a different number of ranks",
                  file=sys.stderr)
            return 2
        return None
    if gpus == 1:
        return None
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def ranks_probe():
    """--ranks-probe: the ranks this invocation runs, gathered over gloo (CPU only), one JSON line
    from rank 0 with the same n_gpus the bench line would carry."""
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    ranks = [rank]
    if world > 1:
        dist.init_process_group("gloo")
        t = torch.tensor([rank, int(os.environ.get("LOCAL_RANK", "0")), os.getpid()], dtype=torch.int64)
        lst = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(lst, t)
        ranks = [int(v[0]) for v in lst]
        pids = len({int(v[2]) for v in lst})
        dist.destroy_process_group()
    else:
        pids = 1
    if rank == 0:
        print(json.dumps({"probe": True, "n_gpus": gpu_fields(world)["n_gpus"], "world": world, "ranks": ranks,
                          "processes": pids}), flush=True)
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=20.0)
    ap.add_argument("--config4-pairs", type=int, default=512, help="0 = skip the configs[3] batch field")
    ap.add_argument("--no-10k", action="store_true", help="skip the configs[1] full-matrix field")
    ap.add_argument("--no-100k-full", action="store_true", help="skip the 100k x 100k full-matrix field")
    ap.add_argument("--no-rank-share", action="store_true", help="skip the config4_rank_share field")
    ap.add_argument("--full-batch-pairs", type=int, default=64, help="0 = skip the full-matrix batch field")
    ap.add_argument("--no-config5", action="store_true", help="skip the configs[4] score-only field")
    ap.add_argument("--config5-cpu-sample", type=int, default=50000, help="n x n prefix for the config-5 CPU leg")
    ap.add_argument("--ranks-probe", action="store_true",
                    help="test aid: start the ranks (gloo), gather them and print the n_gpus/ranks line; no GPU")
    a = ap.parse_args()

    code = launch_ranks(a.gpus)  # before anything touches the GPU
    if code is not None:
        sys.exit(code)

    import torch
    import torch.distributed as dist
    if a.ranks_probe:
        sys.exit(ranks_probe())
    import gpuseqalign_amd as gsa

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if REHEARSE:
        local = 0
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("gloo" if REHEARSE else "nccl")
    dev = torch.device("cuda", local if world > 1 else 0)

    sub = subst_blosum62()
    tS = torch.from_numpy(sub).to(coll_dev(dev))
    if world > 1:
        dist.broadcast(tS, src=0)  # substitution table from rank 0 (RCCL over xGMI)
    tS = tS.to(dev)
    eng = gsa.Engine(dev.index)
    stream = torch.cuda.Stream(device=dev)
    sh = stream.cuda_stream

    # ---- headline: config 3, 100k x 100k sparse fill --------------------------------------
    Y, X = config3_pair()
    R, C = len(Y) - 1, len(X) - 1
    tY, tX = torch.from_numpy(Y).to(dev), torch.from_numpy(X).to(dev)
    geom = gsa.sparse_geometry(R + 1, C + 1, TILE_BX)
    hrow = torch.empty(geom.hrowElems, dtype=torch.int32, device=dev)
    hcol = torch.empty(geom.hcolElems, dtype=torch.int32, device=dev)

    def step():
        eng.fill_sparse_dev(tY.data_ptr(), R + 1, tX.data_ptr(), C + 1, tS.data_ptr(), 25, -11, TILE_BX,
                            hrow.data_ptr(), hcol.data_ptr(), sh)

    elapsed, kern_ms = timed_steps(step, stream, dev, a.steps, a.warmup, world, eng)
    # align_cost as the reference's mlsp align computes it (recompute of the last tile from its
    # headers, nwalign_gpu9_mlsp_diagdiagdiag.cu:713-716): only the last tile's headers come back
    last = geom.tileHdrMatRows * geom.tileHdrMatCols - 1
    hr = np.zeros(geom.hrowElems, dtype=np.int32)
    hc = np.zeros(geom.hcolElems, dtype=np.int32)
    hr[last * geom.tileHrowLen:] = hrow[last * geom.tileHrowLen:].cpu().numpy()
    hc[last * geom.tileHcolLen:] = hcol[last * geom.tileHcolLen:].cpu().numpy()
    cost = gsa.sparse_align_cost(gsa.SparseResult(hr, hc, geom, 0, {}), Y, X, sub, -11)
    del hr, hc
    costs = [cost]
    if world > 1:
        t = torch.tensor([cost], dtype=torch.int64, device=coll_dev(dev))
        lst = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(lst, t)
        costs = [int(v.item()) for v in lst]
    gold = load_golden("config3_100k.json")
    gold_cost = None if gold is None else gold["pairs"]["related"]["align_cost"]

    cells = float(R) * float(C)
    value = world * cells * a.steps / elapsed / 1e9
    ops_achieved = OPS_PER_CELL * cells / (kern_ms * 1e-3) / 1e12
    hdr_bytes = 4.0 * (geom.hrowElems + geom.hcolElems)
    kname = sparse_kernel_name()
    del hrow, hcol
    torch.cuda.empty_cache()

    # ---- configs[1]: 10k x 10k full matrix (secondary field) ------------------------------
    full10k = None
    if not a.no_10k:
        Y2, X2 = config2_pair()
        R2, C2 = len(Y2) - 1, len(X2) - 1
        tY2, tX2 = torch.from_numpy(Y2).to(dev), torch.from_numpy(X2).to(dev)
        score = torch.empty((R2 + 1) * (C2 + 1), dtype=torch.int32, device=dev)

        def step2():
            eng.fill_full_dev(tY2.data_ptr(), R2 + 1, tX2.data_ptr(), C2 + 1, tS.data_ptr(), 25, -11,
                              score.data_ptr(), sh)

        el2, km2 = timed_steps(step2, stream, dev, a.steps, a.warmup, world, eng)
        b2 = 4.0 * (R2 + 1) * (C2 + 1)
        full10k = {"workload": "BASELINE configs[1]: NW-LG len12124[:10000] x len15390[:10000] "
                               "(resrc/seq_generated.fa), full int32 score matrix in HBM",
                   "value": round(world * R2 * C2 * a.steps / el2 / 1e9, 2), "unit": "GCUPS",
                   "ms_per_step": round(el2 * 1e3 / a.steps, 4), "kernel_ms": round(km2, 4),
                   "kernel": full_kernel_name(True),
                   "hbm_write_GBps": round(b2 / (km2 * 1e-3) / 1e9, 1),
                   "hbm_frac": round(b2 / (km2 * 1e-3) / 1e9 / PEAK_HBM_GBPS, 4),
                   "align_cost": int(score[-1].item()), "golden_align_cost": -4922,
                   "critical_path": (critical_path(C2, -(-R2 // (64 * lane_ns())) * lane_ns(), 4, km2, 64)
                                     if os.environ.get("GSA_FULL_KERNEL", "") == "lane" else
                                     critical_path(C2, -(-R2 // 256), 9, km2, 256))}
        del score
        torch.cuda.empty_cache()
    # ---- the headline pair as a full matrix (40 GB) ----------------------------------------
    full100k = None
    if not a.no_100k_full:
        full100k = bench_full100k(dev, eng, tS, sh, stream, max(3, a.steps // 4), 2, world)
    cfg5 = None
    if not a.no_config5:
        cfg5 = bench_config5(dev, eng, max(3, a.steps // 4), 2, 0 if a.no_cpu_baseline else a.config5_cpu_sample,
                             rank, world)
    eng.sync(sh)
    eng.close()
    torch.cuda.empty_cache()

    # ---- full-matrix family at throughput (HBM-write bound) ------------------------------
    fullb = bench_full_batch(world, rank, local, a.full_batch_pairs) if a.full_batch_pairs > 0 else None
    torch.cuda.empty_cache()

    # ---- configs[3]: 512 pairs, LPT-sharded (strong scaling field) ------------------------
    cfg4 = bench_config4(world, rank, local, a.config4_pairs) if a.config4_pairs > 0 else None
    share = None
    if a.config4_pairs > 0 and world == 1 and not REHEARSE and not a.no_rank_share:
        share = bench_config4_rank_share(local, a.config4_pairs, cfg4)

    if rank == 0:
        gf = gpu_fields(world)
        out = {
            "metric": METRIC, "value": round(value, 3), "unit": "GCUPS", "n_gpus": gf["n_gpus"], "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(elapsed * 1e3 / a.steps, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "int32",
            "data": "synthetic (splitmix64: seqX seed 100, seqY = seqX mutated seed 101); blosum62, gapo -11",
            "config": {"workload": f"BASELINE configs[2]: NW-LG {R}x{C} related pair, sparse tile-header (mlsp) "
                                   f"fill, tileBx {TILE_BX} x tileBy {geom.tileHcolLen - 1}, headers only in HBM",
                       "R": R, "C": C, "pairs_per_rank": 1, "representation": "sparse tile headers (mlsp)",
                       "parallelism": gf["parallelism"]},
            "rehearsal": gf["rehearsal"],
            "roofline": {"bound": "valu", "achieved": round(ops_achieved, 3), "peak": round(PEAK_VALU_TOPS, 2),
                         "unit": "T int32 lane-ops/s", "frac": round(ops_achieved / PEAK_VALU_TOPS, 4),
                         "traffic": traffic_for("traffic_config3.json", R, C, kname),
                         "kernel": kname, "kernel_ms": round(kern_ms, 4), "ops_per_cell": OPS_PER_CELL,
                         "algorithmic_ops_per_launch": OPS_PER_CELL * cells,
                         "header_bytes_per_launch": hdr_bytes,
                         "header_GBps": round(hdr_bytes / (kern_ms * 1e-3) / 1e9, 1),
                         "hbm_frac": round(hdr_bytes / (kern_ms * 1e-3) / 1e9 / PEAK_HBM_GBPS, 5),
                         "critical_path": critical_path(C, -(-R // 256), 9, kern_ms, 256)},
            "align_costs": costs[:8], "golden_align_cost": gold_cost,
            "golden_match": None if gold_cost is None else all(c == gold_cost for c in costs),
            "fill_10k_full": full10k, "fill_100k_full": full100k, "config4": cfg4, "config4_rank_share": share, "full_batch": fullb, "config5": cfg5,
        }
        if not a.no_cpu_baseline and world == 1:  # the CPU leg runs on rank 0 at N = 1 only
            out["cpu_baseline"] = cpu_baseline(Y, X, sub, budget_s=a.cpu_budget)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
