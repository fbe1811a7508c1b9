"""Stamp timeline of the fused single-pair full fill on the configs[1] 10k pair:
GSA_STAMPS=1 makes the kernel record s_memrealtime (100 MHz) at every pass-1 strip's start and end
and at every expansion task's claim, readiness and end (gsa_debug_stamps).  Prints one JSON summary:
the lag between consecutive strips inside a ticket and across tickets (the wavefront's hop), strip
durations, task waits and durations, and the tail from the last strip's end to the last task's end.
Cycles are at 2.4 GHz (24 per stamp tick)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np


def main():
    os.environ["GSA_STAMPS"] = "1"
    os.environ.setdefault("GSA_FULL_FUSED", "1")
    import torch
    import gpuseqalign_amd as gsa
    import bench

    dev = torch.device("cuda:0")
    Y, X = bench.config2_pair()
    sub = bench.subst_blosum62()
    y, x, s = (torch.from_numpy(np.ascontiguousarray(v, dtype=np.int32)).to(dev) for v in (Y, X, sub))
    eng = gsa.Engine(0)
    R1, C1 = len(Y), len(X)
    ld = gsa.full_pitch(C1)
    buf = torch.empty(R1 * ld + 64, dtype=torch.int32, device=dev)
    ptr = buf.data_ptr() + 4 * gsa.full_base_offset()
    runs = []
    for rep in range(4):
        eng.fill_full_dev(y.data_ptr(), R1, x.data_ptr(), C1, s.data_ptr(), 25, -11, ptr, ld=ld)
        eng.sync()
        st = eng.debug_stamps().astype(np.int64)
        if rep:
            runs.append(st)
    ok = int(buf[gsa.full_base_offset() + (R1 - 1) * ld + C1 - 1].item()) == -4922
    ns = 4
    tickets = -(-(R1 - 1) // 1024)
    nstrips = tickets * ns
    out = []
    for st in runs:
        strips = st[:2 * nstrips].reshape(nstrips, 2)  # [ticket start, strip end]
        tasks = st[2 * nstrips:].reshape(-1, 3)
        t0 = min(strips[:, 0].min(), tasks[tasks[:, 0] > 0, 0].min())
        cyc = 24.0
        start = (strips[:, 0] - t0) * cyc
        end = (strips[:, 1] - t0) * cyc
        lag = np.diff(end)  # strips end in wavefront order, spaced by the lag
        intra = [lag[i - 1] for i in range(1, nstrips) if i % ns]
        inter = [lag[i - 1] for i in range(1, nstrips) if i % ns == 0]
        wait = (tasks[:, 1] - tasks[:, 0]) * cyc
        dur = (tasks[:, 2] - tasks[:, 1]) * cyc
        out.append({
            "kernel_span_us": round(float((tasks[:, 2].max() - t0) / 100.0), 2),
            "last_strip_end_us": round(float(end.max() / cyc / 100.0), 2),
            "tail_after_last_strip_us": round(float((tasks[:, 2].max() - strips[:, 1].max()) / 100.0), 2),
            "strip_lag_intra_cycles_median": round(float(np.median(intra)), 0),
            "strip_lag_inter_cycles_median": round(float(np.median(inter)), 0),
            "strip_lag_inter_cycles": [round(float(v), 0) for v in inter],
            "lag_per_256_rows_cycles_mean": round(float(np.mean(lag)), 0),
            "strip_duration_from_ticket_start_cycles_median": round(float(np.median(end - start)), 0),
            "task_wait_cycles_median": round(float(np.median(wait)), 0),
            "task_duration_cycles_median": round(float(np.median(dur)), 0),
            "tasks": int(len(tasks)), "strips": int(nstrips),
        })
    print(json.dumps({"workload": "configs[1] 10k x 10k full fill, fused two-pass kernel, pitched layout",
                      "align_cost_ok": ok, "runs": out}, indent=1))
    eng.close()


if __name__ == "__main__":
    main()
