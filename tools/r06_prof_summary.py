"""Summaries of tools/r06_prof.sh's output (gpurun_out/TAG) into profiles/: the kernel-stats rows,
the full batch's timed launches from the kernel trace (one row per pass), and the WRITE_SIZE /
FETCH_SIZE passes per workload against the algorithmic bytes (units kB -> bytes x 1024; FETCH_SIZE
is doubled for the wide streaming loads the guide calibrates, and reported raw beside it)."""
import csv
import collections
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def counters(d, ctr, key):
    agg, names = collections.defaultdict(float), {}
    for r in csv.DictReader(open(os.path.join(d, f"{ctr}/run_counter_collection.csv"))):
        if key in r["Kernel_Name"]:
            k = int(r["Dispatch_Id"])
            agg[k] += float(r["Counter_Value"])
            names[k] = r["Kernel_Name"]
    last = max(agg)
    return agg[last] * 1024.0, names[last]


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r06prof"
    src = os.path.join(ROOT, "gpurun_out", tag)
    prof = os.path.join(ROOT, "profiles")
    for part, name in (("A", "headline"), ("B", "full100k"), ("C", "full_batch")):
        shutil.copy(os.path.join(src, part, "run_kernel_stats.csv"), os.path.join(prof, f"r06_{name}_kernel_stats.csv"))
    # the batch: the last three launches (the timed ones, after the tuner's candidates)
    rows = [r for r in csv.DictReader(open(os.path.join(src, "C", "run_kernel_trace.csv")))
            if "nw_expand_stream_kernel" in r["Kernel_Name"] or "nw_krow_kernel<8, 4, 1024, 2, true>" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    tail = rows[-6:]
    p1 = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in tail if "krow" in r["Kernel_Name"]]
    p2 = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in tail if "expand" in r["Kernel_Name"]]
    from gpuseqalign_amd import shard
    pairs = shard.synthetic_batch(64, 18000, 22000, seed0=1000)
    alg_batch = 4.0 * sum(len(y) * len(x) for y, x in pairs)
    import bench
    Y, X = bench.config3_pair()
    alg_full = 4.0 * len(Y) * len(X)
    out = {"source": f"tools/r06_prof.sh on one MI355X (gpurun), round 6; summarised by tools/r06_prof_summary.py",
           "full_batch_timed_launches": {
               "workload": "64 NW-LG pairs (18-22k, seeds 1000+k), full int32 matrices, pitched; tools/batch_bench.py "
                           "--mode full --pairs 64 --warmup 6 --repeats 3 (the bench's full_batch field)",
               "pass1_kernel": "nw_krow_kernel<8, 4, 1024, 2, true>", "pass1_ms": [round(v, 4) for v in p1],
               "pass2_kernel": "nw_expand_stream_kernel", "pass2_ms": [round(v, 4) for v in p2],
               "launch_ms_mean": round((sum(p1) + sum(p2)) / max(1, len(p2)), 4),
               "algorithmic_write_bytes": alg_batch,
               "hbm_frac_of_kernel_time": round(alg_batch / ((sum(p1) + sum(p2)) / len(p2) * 1e-3) / 8e12, 4)}}
    pmc = {}
    for tagw, key, alg in (("h", "nw_krow_kernel<4, 4, 1024, 0, true>", None),
                           ("f", "nw_full_fused_kernel<4, 8, true", alg_full),
                           ("b1", "nw_krow_kernel<8, 4, 1024, 2, true>", None),
                           ("b2", "nw_expand_stream_kernel", alg_batch)):
        d = os.path.join(src, tagw[0] + "_")
        wr, name = counters(src, f"{tagw[0]}_WRITE_SIZE", key)
        fe, _ = counters(src, f"{tagw[0]}_FETCH_SIZE", key)
        pmc[tagw] = {"kernel": name, "write_bytes": wr, "fetch_bytes_raw": fe, "fetch_bytes_x2": 2 * fe}
        if alg:
            pmc[tagw]["algorithmic_write_bytes"] = alg
            pmc[tagw]["write_over_algorithmic"] = round(wr / alg, 4)
    wb = pmc["b1"]["write_bytes"] + pmc["b2"]["write_bytes"]
    pmc["batch_both_passes"] = {"write_bytes": wb, "write_over_algorithmic": round(wb / alg_batch, 4)}
    out["pmc"] = pmc
    json.dump(out, open(os.path.join(prof, "r06_pmc.json"), "w"), indent=1)
    # the bench's full_batch field reads its PMC write ratio from here
    json.dump({"workload": out["full_batch_timed_launches"]["workload"],
               "kernel": "gsa::nw_krow_kernel<8,4,1024,2,true> (pass 1) + gsa::nw_expand_stream_kernel (pass 2)",
               "write_bytes": wb, "algorithmic_write_bytes": alg_batch,
               "write_over_algorithmic": round(wb / alg_batch, 4),
               "pass2_write_over_algorithmic": pmc["b2"]["write_over_algorithmic"],
               "source": "profiles/r06_pmc.json (tools/r06_prof.sh, WRITE_SIZE pass over one launch)"},
              open(os.path.join(prof, "r06_pmc_full_batch.json"), "w"), indent=1)
    # the headline's traffic (bench roofline.traffic)
    h = pmc["h"]
    tj = json.load(open(os.path.join(prof, "traffic_config3.json")))
    tj.update({"hbm_bytes_per_launch": int(h["write_bytes"] + h["fetch_bytes_raw"]), "write_bytes": int(h["write_bytes"]),
               "read_bytes": int(h["fetch_bytes_raw"]),
               "method": "rocprofv3 --pmc WRITE_SIZE and FETCH_SIZE in separate passes (tools/r06_prof.sh), last dispatch of "
                         "the int8-profile instance; kB units -> bytes x1024. FETCH_SIZE is not doubled: the guide's 1/2 "
                         "correction is for 16-B-per-lane streaming reads, and these are 8-B-per-lane granule loads",
               "source": "profiles/r06_pmc.json (round 6)"})
    json.dump(tj, open(os.path.join(prof, "traffic_config3.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
