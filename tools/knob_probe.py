"""Timing probe across GSA_KNOB experiment builds: one process per library (GSA_LIB)."""
import os, subprocess, sys, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
libs = sys.argv[1:] or ["libgsa.so"]
code = r'''
import sys, json; sys.path.insert(0, "%s")
import gpuseqalign_amd as gsa
from tools.gpu_perf import run
eng = gsa.Engine(0)
for R, C, mode, tbx in [(256, 20000, "sparse", 256), (256, 20000, "sparse", 4096), (256, 20000, "full", 256), (10000, 10000, "full", 256)]:
    r = run(eng, R, C, mode, tbx, reps=3)
    steps = C + 64
    print(json.dumps({"lib": "%s", "R": R, "C": C, "mode": mode, "tBx": tbx, "ms": round(r["ms"], 4), "cyc_per_step@2.4GHz": round(r["ms"] * 2.4e6 / steps, 1)}))
'''
for lib in libs:
    env = dict(os.environ, GSA_LIB=os.path.join(ROOT, "gpuseqalign_amd", lib))
    out = subprocess.run([sys.executable, "-c", code % (ROOT, lib)], env=env, capture_output=True, text=True, timeout=120)
    print(out.stdout.strip() or out.stderr[-2000:], flush=True)
