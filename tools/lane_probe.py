"""Lane-kernel timing probe: full fills of R x C for a ladder of R (hop cost per strip), per
strips-per-workgroup count (GSA_LANE_NS is read per launch)."""
import os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gpuseqalign_amd as gsa
from tools.gpu_perf import run

eng = gsa.Engine(0)
C = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
rows = [int(x) for x in os.environ.get("ROWS", "64,128,256,512,1024,2048,4096,10000").split(",")]
for kern, nss in (("lane", tuple(int(x) for x in os.environ.get("NSS", "1,2,3,4").split(","))),):
    for ns in nss:
        os.environ["GSA_LANE_NS"] = str(ns)
        prev = None
        for R in rows:
            r = run(eng, R, C, "full", reps=5)
            cyc = r["ms"] * 2.4e6
            rec = {"kernel": kern, "ns": ns, "R": R, "C": C, "ms": round(r["ms"], 4), "cyc_per_step": round(cyc / (C + 64), 1)}
            if prev is not None:
                # extra cycles per extra 64 rows, in units of the single-strip step
                rec["hop_cyc_per_64rows"] = round((cyc - prev[1]) / ((R - prev[0]) / 64), 0)
            prev = (R, cyc)
            print(json.dumps(rec), flush=True)
