"""Summarise rocprofv3 --pmc output directories (p*/run_counter_collection.csv): per-counter value of the LAST fill dispatch (kernel name
containing argv[2], default nw_lane|nw_strip)."""
import csv, collections, glob, json, sys
out = {}
keys = sys.argv[2].split("|") if len(sys.argv) > 2 else ["nw_lane", "nw_strip"]
for f in sorted(glob.glob(sys.argv[1] + "/p*/run_counter_collection.csv")):
    agg = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        if any(k in r["Kernel_Name"] for k in keys):
            agg[(int(r["Dispatch_Id"]), r["Counter_Name"])] += float(r["Counter_Value"])
    if not agg:
        continue
    last = max(d for d, _ in agg)
    for (d, c), v in agg.items():
        if d == last:
            out[c] = v
print(json.dumps(out, indent=1))
