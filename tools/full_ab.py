"""Full-matrix fill timing, unpadded vs pitched device layout (gsa_full_pitch), same process:
the configs[1] 10k pair (two-pass fill fused into one launch, and in two: GSA_FULL_FUSED) and
optionally a configs[3]-shaped batch.  Each result's
last cell is checked against the known align_cost (-4922) / the first pass.  JSON lines."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--batch", type=int, default=64, help="pairs of the batch leg (0 = skip)")
    ap.add_argument("--no-10k", action="store_true")
    ap.add_argument("--variants", nargs="*", default=[],
                    help="batch leg (pitched) once per variant, each 'NAME=V,NAME=V' environment settings "
                         "(read per launch); default: unpadded vs pitched")
    a = ap.parse_args()
    import torch
    import gpuseqalign_amd as gsa
    from gpuseqalign_amd import shard
    import bench

    dev = torch.device("cuda:0")
    Y, X = bench.config2_pair()
    sub = bench.subst_blosum62()
    y, x, s = (torch.from_numpy(np.ascontiguousarray(v, dtype=np.int32)).to(dev) for v in (Y, X, sub))
    eng = gsa.Engine(0)
    st = torch.cuda.Stream(device=dev)
    R1, C1 = len(Y), len(X)
    for rnd in range(a.rounds):
        for pitched, fused in (() if a.no_10k else ((False, "1"), (True, "0"), (True, "1"))):
            os.environ["GSA_FULL_FUSED"] = fused  # read per launch
            ld = gsa.full_pitch(C1) if pitched else C1
            off = gsa.full_base_offset() if pitched else 0
            buf = torch.empty(R1 * ld + 64, dtype=torch.int32, device=dev)
            ptr = buf.data_ptr() + 4 * off

            def run():
                eng.fill_full_dev(y.data_ptr(), R1, x.data_ptr(), C1, s.data_ptr(), 25, -11, ptr, st.cuda_stream,
                                  ld=ld if pitched else None)
            for _ in range(3):
                run()
            eng.sync(st.cuda_stream)
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.reps)]
            with torch.cuda.stream(st):
                for e0, e1 in evs:
                    e0.record(st)
                    run()
                    e1.record(st)
            eng.sync(st.cuda_stream)
            torch.cuda.synchronize()
            ms = float(np.median([e0.elapsed_time(e1) for e0, e1 in evs]))
            cost = int(buf[off + (R1 - 1) * ld + C1 - 1].item())
            print(json.dumps({"leg": "10k", "pitched": pitched, "fused": fused == "1", "ld": ld, "kernel_ms": round(ms, 4),
                              "gcups": round((R1 - 1) * (C1 - 1) / ms / 1e6, 2), "align_cost": cost,
                              "ok": cost == -4922}), flush=True)
            del buf
        if a.batch > 0:
            pairs = shard.synthetic_batch(a.batch, 18000, 22000, seed0=1000)
            ref = None
            legs = [(True, v) for v in a.variants] if a.variants else [(False, ""), (True, "")]
            for pitched, var in legs:
                for kv in filter(None, var.split(",")):
                    k, v = kv.split("=")
                    os.environ[k] = v
                torch.cuda.empty_cache()
                fn = shard.gpu_batch_align(0, mode="full", warmup=1, repeats=3, pitched=pitched,
                                           out_budget_bytes=int(0.9 * 140e9))
                costs, secs = fn(list(range(len(pairs))), pairs, sub, -11)
                cells = sum((len(p[0]) - 1) * (len(p[1]) - 1) for p in pairs)
                ref = costs if ref is None else ref
                for kv in filter(None, var.split(",")):
                    os.environ.pop(kv.split("=")[0], None)
                print(json.dumps({"leg": f"batch{a.batch}", "pitched": pitched, "variant": var, "seconds": round(secs, 5),
                                  "gcups": round(cells / secs / 1e9, 2),
                                  "matrix_TBps": round(4 * sum(len(p[0]) * len(p[1]) for p in pairs) / secs / 1e12, 3),
                                  "costs_equal_first": costs == ref}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
