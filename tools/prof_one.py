"""Run one fill configuration a few times (for rocprofv3 sessions)."""
import os, sys, argparse
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import gpuseqalign_amd as gsa
from tools.gpu_perf import run

ap = argparse.ArgumentParser()
ap.add_argument("--R", type=int, default=252)
ap.add_argument("--C", type=int, default=20000)
ap.add_argument("--mode", default="sparse")
ap.add_argument("--tileBx", type=int, default=256)
ap.add_argument("--reps", type=int, default=3)
a = ap.parse_args()
eng = gsa.Engine(0)
print(run(eng, a.R, a.C, a.mode, a.tileBx, reps=a.reps))
