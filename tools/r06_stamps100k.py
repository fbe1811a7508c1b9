"""Stamp timeline of the fused full fill on the config-3 100k x 100k pair (pitched, 40 GB):
GSA_STAMPS=1 (pass-1 strip start/end, expansion task claim/ready/done, s_memrealtime 100 MHz).
Saves the raw stamps of the last run to gpurun_out/r06_stamps100k<tag>.npz and prints a summary:
pass-1 strip ends, task waits and durations, and the expansion's completed bytes per 0.5 ms."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else ""
    ten = "10k" in sys.argv[2:]
    os.environ["GSA_STAMPS"] = "1"
    import torch
    import gpuseqalign_amd as gsa
    import bench

    dev = torch.device("cuda:0")
    Y, X = bench.config2_pair() if ten else bench.config3_pair()
    sub = bench.subst_blosum62()
    y, x, s = (torch.from_numpy(np.ascontiguousarray(v, dtype=np.int32)).to(dev) for v in (Y, X, sub))
    eng = gsa.Engine(0)
    R1, C1 = len(Y), len(X)
    ld = gsa.full_pitch(C1)
    buf = torch.empty(R1 * ld + 64, dtype=torch.int32, device=dev)
    ptr = buf.data_ptr() + 4 * gsa.full_base_offset()
    for rep in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        eng.fill_full_dev(y.data_ptr(), R1, x.data_ptr(), C1, s.data_ptr(), 25, -11, ptr, ld=ld)
        e1.record()
        eng.sync()
        ms = e0.elapsed_time(e1)
        st = eng.debug_stamps().astype(np.int64)
    ok = int(buf[gsa.full_base_offset() + (R1 - 1) * ld + C1 - 1].item()) == (-4922 if ten else 450138)
    ns = 4
    tickets = -(-(R1 - 1) // 1024)
    nstrips = tickets * ns
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.savez_compressed(os.path.join(ROOT, "gpurun_out", f"r06_stamps100k{tag}.npz"), st=st, nstrips=nstrips)
    strips = st[:4 * nstrips].reshape(nstrips, 4)
    tasks = st[4 * nstrips:].reshape(-1, 3)
    t0 = min(strips[:, 0].min(), tasks[tasks[:, 0] > 0, 0].min())
    us = lambda v: (v - t0) / 100.0
    end = us(strips[:, 1])
    wait = (tasks[:, 1] - tasks[:, 0]) / 100.0
    dur = (tasks[:, 2] - tasks[:, 1]) / 100.0
    done = us(tasks[:, 2])
    bw = 50 if ten else 500
    bins = np.arange(0, done.max() + bw, bw)
    hist, _ = np.histogram(done, bins=bins)
    out = {"ms": round(ms, 4), "cost_ok": ok, "strips": int(nstrips), "tasks": int(len(tasks)),
           "span_us": round(float(done.max()), 1),
           "strip_end_us": {"first": round(float(end.min()), 1), "median": round(float(np.median(end)), 1),
                            "last": round(float(end.max()), 1)},
           "strip_start_us_last": round(float(us(strips[:, 0]).max()), 1),
           "strip_clock_ghz": {"first": round(float((strips[0, 3] - strips[0, 2]) / ((strips[0, 1] - strips[0, 0]) * 10.0)), 3),
                               "median": round(float(np.median((strips[:, 3] - strips[:, 2]) /
                                                               ((strips[:, 1] - strips[:, 0]) * 10.0))), 3)},
           "task_wait_us": {"median": round(float(np.median(wait)), 2), "p90": round(float(np.percentile(wait, 90)), 2),
                            "sum_ms": round(float(wait.sum()) / 1e3, 2)},
           "task_dur_us": {"median": round(float(np.median(dur)), 2), "p10": round(float(np.percentile(dur, 10)), 2),
                           "p90": round(float(np.percentile(dur, 90)), 2), "sum_ms": round(float(dur.sum()) / 1e3, 2)},
           f"tasks_done_per_{bw}us": hist.tolist(),
           "first_claim_us": round(float(us(tasks[:, 0]).min()), 1)}
    print(json.dumps(out), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
