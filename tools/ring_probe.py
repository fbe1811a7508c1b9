"""Ring-mode full fills: timing per library (GSA_LIB) and env (GSA_FULL_RING), one process each."""
import os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
code = r'''
import sys, json; sys.path.insert(0, "%s")
import numpy as np
import gpuseqalign_amd as gsa
from tools.gpu_perf import run
from tests._data import random_pair, Golden
eng = gsa.Engine(0)
for R, C in [(10000, 10000), (23728, 23728), (4097, 3001)]:
    r = run(eng, R, C, "full", reps=5)
    print(json.dumps({"tag": "%s", "R": R, "C": C, "ms": round(r["ms"], 4), "gcups": round(r["gcups"], 1)}), flush=True)
G = Golden(); Y, X = random_pair(4097, 3001, 5)
import oracle
S, c = oracle.fill_full(Y, X, G.blosum62, -11)
print(json.dumps({"tag": "%s", "parity_4097x3001": bool(np.array_equal(eng.align_full(Y, X, G.blosum62, -11).score, S))}))
'''
for spec in sys.argv[1:]:
    lib, ring = spec.split(":")
    env = dict(os.environ, GSA_LIB=os.path.join(ROOT, "gpuseqalign_amd", lib), GSA_FULL_RING=ring)
    tag = spec
    out = subprocess.run([sys.executable, "-c", code % (ROOT, tag, tag)], env=env, capture_output=True, text=True, timeout=200)
    print(out.stdout.strip() or out.stderr[-2000:], flush=True)
