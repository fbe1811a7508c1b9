"""Lane-kernel knob probe: one process per GSA_LKNOB build (GSA_LIB), single strip and 10k."""
import os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
libs = sys.argv[1:] or ["libgsa.so"]
code = r'''
import sys, json, os; sys.path.insert(0, "%s")
import gpuseqalign_amd as gsa
from tools.gpu_perf import run
eng = gsa.Engine(0)
for ns in (1, 2):
    os.environ["GSA_LANE_NS"] = str(ns)
    for R, C in [(64, 10000), (128, 10000), (1024, 10000), (10000, 10000)]:
        r = run(eng, R, C, "full", reps=3)
        print(json.dumps({"lib": "%s", "ns": ns, "R": R, "C": C, "ms": round(r["ms"], 4), "cyc_per_step": round(r["ms"] * 2.4e6 / (C + 64), 1)}))
'''
for lib in libs:
    env = dict(os.environ, GSA_LIB=os.path.join(ROOT, "gpuseqalign_amd", lib))
    out = subprocess.run([sys.executable, "-c", code % (ROOT, lib)], env=env, capture_output=True, text=True, timeout=120)
    print(out.stdout.strip() or out.stderr[-2000:], flush=True)
