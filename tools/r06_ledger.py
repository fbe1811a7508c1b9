"""(Needs a ledger build: tools/r06_variant_build.sh led -DGSA_KR_LEDGER=1 "nw_krow.hip nw_krowx.hip", run with
GSA_LIB=gpuseqalign_amd/libgsa_led.so; -DGSA_KR_BLOCK_LEDGER=1 adds the block spans.)
Cycle ledger of the headline K-rows sparse fill (config-3 100k x 100k pair, nw_krow_kernel<4,4,...>)
under GSA_STAMPS=1: per strip the real-time and shader-clock span and the cycles spent waiting for
input (the spin path); prints the ledger as JSON and saves the raw words under gpurun_out/.
Usage: python tools/r06_ledger.py [R C] [xr] (default: the config-3 pair; R C: a prefix of it; xr: the
two-pass full fill's pass 1 instead, GSA_FULL_FUSED=0, into a pitched matrix)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np


def main():
    os.environ["GSA_STAMPS"] = "1"
    import torch
    import gpuseqalign_amd as gsa
    import bench
    Y, X = bench.config3_pair()
    xr = "xr" in sys.argv[1:]
    args = [v for v in sys.argv[1:] if v != "xr"]
    if len(args) > 1:
        Y, X = Y[:int(args[0]) + 1], X[:int(args[1]) + 1]
    if xr:
        os.environ["GSA_FULL_FUSED"] = "0"
    R, C = len(Y) - 1, len(X) - 1
    dev = torch.device("cuda:0")
    sub = bench.subst_blosum62()
    tY, tX, tS = (torch.from_numpy(np.ascontiguousarray(v, dtype=np.int32)).to(dev) for v in (Y, X, sub))
    geom = gsa.sparse_geometry(R + 1, C + 1, bench.TILE_BX)
    hrow = torch.empty(geom.hrowElems, dtype=torch.int32, device=dev)
    hcol = torch.empty(geom.hcolElems, dtype=torch.int32, device=dev)
    eng = gsa.Engine(0)
    if xr:
        ld = gsa.full_pitch(C + 1)
        mat = torch.empty((R + 1) * ld + gsa.full_base_offset() + 64, dtype=torch.int32, device=dev)
        base = mat.data_ptr() + 4 * gsa.full_base_offset()
    ms = []
    for rep in range(4):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        if xr:
            eng.fill_full_dev(tY.data_ptr(), R + 1, tX.data_ptr(), C + 1, tS.data_ptr(), 25, -11, base, ld=ld)
        else:
            eng.fill_sparse_dev(tY.data_ptr(), R + 1, tX.data_ptr(), C + 1, tS.data_ptr(), 25, -11, bench.TILE_BX,
                                hrow.data_ptr(), hcol.data_ptr())
        e1.record()
        eng.sync()
        ms.append(e0.elapsed_time(e1))
    st = eng.debug_stamps().astype(np.int64).reshape(-1, 10)
    if not st[:, 1].any():
        sys.exit("no ledger stamps: run a GSA_KR_LEDGER build (see the docstring)")
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.save(os.path.join(ROOT, "gpurun_out", f"r06_ledger_{R}x{C}{'_xr' if xr else ''}.npy"), st)
    st = st[st[:, 1] > 0]
    rt0 = st[:, 0].min()
    start = (st[:, 0] - rt0) / 100.0  # us
    end = (st[:, 1] - rt0) / 100.0
    span_us = end - start
    cyc = (st[:, 3] - st[:, 2]).astype(np.float64)
    clk = cyc / (span_us * 1e3)  # GHz
    spin = st[:, 4].astype(np.float64)
    nblk = (C + 65 + 15) // 16
    busy = cyc - spin
    out = {"R": R, "C": C, "mode": "xr pass 1" if xr else "sparse", "ms": [round(v, 4) for v in ms[1:]], "strips": int(len(st)),
           "first_strip": {"start_us": round(float(start[0]), 2), "end_us": round(float(end[0]), 2),
                           "span_us": round(float(span_us[0]), 1), "clock_ghz": round(float(clk[0]), 3),
                           "wait_frac": round(float(spin[0] / cyc[0]), 4), "waits": int(st[0, 5]),
                           "busy_cycles_per_step": round(float(busy[0] / (16 * nblk)), 2)},
           "last_strip_end_us": round(float(end.max()), 1),
           "median": {"span_us": round(float(np.median(span_us)), 1), "clock_ghz": round(float(np.median(clk)), 3),
                      "wait_frac": round(float(np.median(spin / cyc)), 4),
                      "busy_cycles_per_step": round(float(np.median(busy / (16 * nblk))), 2),
                      "waits": int(np.median(st[:, 5]))},
           "strip_start_lag_us": round(float(np.median(np.diff(np.sort(start)))), 3),
           "strip_end_lag_us": round(float(np.median(np.diff(np.sort(end)))), 3)}
    if st[:, 6:].any():
        # GSA_KR_BLOCK_LEDGER build: per-step cycles of the block's spans (input wait + halo read,
        # 16 steps, hand-off and captures, between blocks), first strip and median
        spans = st[:, 6:10].astype(np.float64) / (16 * nblk)
        names = ["wait_and_halo", "steps", "handoff_capture", "between_blocks"]
        out["block_ledger_cycles_per_step"] = {
            "first_strip": {k: round(float(v), 2) for k, v in zip(names, spans[0])},
            "median": {k: round(float(v), 2) for k, v in zip(names, np.median(spans, axis=0))}}
    # the critical path: the last strip's end = the first strip's sweep + the lags
    out["ledger_ms"] = {"first_sweep": round(float(span_us[0]) / 1e3, 4),
                        "lag_total": round(float(end.max() - end[np.argmin(start)]) / 1e3, 4)}
    print(json.dumps(out), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
