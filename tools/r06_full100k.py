#!/usr/bin/env python3
"""Probe: the north star's 100k x 100k NW-LG FULL-matrix fill (config-3 related pair, 40 GB int32)
through gsa_fill_full_dev / gsa_fill_full_pitched_dev.  Times the fill with HIP events on its
stream, reads the corner (align_cost), optionally runs the device full check.
Usage: python tools/r06_full100k.py [--reps N] [--pitched] [--check] [--env K=V ...]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--pitched", action="store_true")
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--hash", action="store_true")
    ap.add_argument("--trace", action="store_true")
    ap.add_argument("--timing", action="store_true")
    ap.add_argument("--tag", default="")
    ap.add_argument("--pair", default="100k", choices=["100k", "10k"], help="10k: BASELINE configs[1]")
    a = ap.parse_args()
    import numpy as np
    import torch
    import bench
    import gpuseqalign_amd as gsa
    Y, X = bench.config2_pair() if a.pair == "10k" else bench.config3_pair()
    sub = bench.subst_blosum62()
    R, C = len(Y) - 1, len(X) - 1
    dev = torch.device("cuda", 0)
    tY, tX = torch.from_numpy(Y).to(dev), torch.from_numpy(X).to(dev)
    tS = torch.from_numpy(sub).to(dev)
    ld = gsa.full_pitch(C + 1) if a.pitched else C + 1
    off = gsa.full_base_offset() if a.pitched else 0
    n = (R + 1) * ld + off + 64
    t0 = time.time()
    buf = torch.empty(n, dtype=torch.int32, device=dev)
    base = buf.data_ptr() + 4 * off
    if a.pitched:
        assert (base + 4) % 128 == 0, "cell (0, 1)... base alignment"
    eng = gsa.Engine(0)
    if a.timing:
        eng.set_full_timing(True)
    st = torch.cuda.Stream(device=dev)
    sh = st.cuda_stream
    out = {"R": R, "C": C, "ld": ld, "pitched": a.pitched, "tag": a.tag, "bytes": 4.0 * (R + 1) * (C + 1)}
    ms = []
    with torch.cuda.stream(st):
        for k in range(a.reps + 1):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            eng.fill_full_dev(tY.data_ptr(), R + 1, tX.data_ptr(), C + 1, tS.data_ptr(), 25, -11, base, sh,
                              ld=ld if a.pitched else None)
            e1.record(st)
            eng.sync(sh)
            if k:
                ms.append(e0.elapsed_time(e1))
            print(f"rep {k}: {e0.elapsed_time(e1):.4f} ms", flush=True)
    out["ms"] = [round(v, 4) for v in ms]
    out["ms_min"] = round(min(ms), 4)
    out["ms_mean"] = round(float(np.mean(ms)), 4)
    out["GBps"] = round(out["bytes"] / (out["ms_mean"] * 1e-3) / 1e9, 1)
    out["hbm_frac"] = round(out["GBps"] / 8000.0, 4)
    out["GCUPS"] = round(R * C / (out["ms_mean"] * 1e-3) / 1e9, 1)
    if a.timing:
        out["timing"] = eng.last_full_timing()
    corner = buf[off + R * ld + C: off + R * ld + C + 1].cpu().numpy()
    out["align_cost"] = int(corner[0])
    g = bench.load_golden("config3_100k.json")
    out["golden_cost"] = -4922 if a.pair == "10k" else g["pairs"]["related"]["align_cost"]
    if a.check and not a.pitched:
        t1 = time.time()
        r = eng.check_full_dev(tY.data_ptr(), R + 1, tX.data_ptr(), C + 1, tS.data_ptr(), 25, -11, base)
        out["check"] = r
        out["check_s"] = round(time.time() - t1, 3)
    if a.check and a.pitched:
        t1 = time.time()
        out["check"] = eng.check_full_dev(tY.data_ptr(), R + 1, tX.data_ptr(), C + 1, tS.data_ptr(), 25, -11, base,
                                          ld=ld)
        out["check_s"] = round(time.time() - t1, 3)
    gr = g["pairs"]["related"]
    if a.trace:
        t1 = time.time()
        th, edit, cost = eng.trace_full_dev(tY.data_ptr(), R + 1, tX.data_ptr(), C + 1, base, ld=ld)
        import hashlib
        out["trace"] = {"hash": "%08x" % th, "golden": gr["trace_hash"], "cost": cost, "len": len(edit),
                        "sha_ok": hashlib.sha256(edit.encode()).hexdigest() == gr["edit_trace_sha256"],
                        "s": round(time.time() - t1, 3)}
    if a.hash:
        t1 = time.time()
        h = eng.hash_full_dev(base, R + 1, C + 1, ld=ld)
        out["hash"] = {"hash": "%08x" % h, "golden": gr["score_hash"], "s": round(time.time() - t1, 3)}
    print(json.dumps(out), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
