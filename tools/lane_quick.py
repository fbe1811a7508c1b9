"""Quick full-fill parity ladder against the oracle (diagnostics): first mismatch per shape."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import gpuseqalign_amd as gsa
import oracle
from tests._data import Golden, random_pair
G = Golden()
eng = gsa.Engine(0)
shapes = [(1, 1), (31, 32), (5, 7), (63, 64), (64, 64), (65, 100), (128, 300), (200, 1100), (1000, 1500), (1100, 2222)]
bad = 0
for R, C in shapes:
    Y, X = random_pair(R, C, R * 31 + C)
    r = eng.align_full(Y, X, G.blosum62, -11)
    S, cost = oracle.fill_full(Y, X, G.blosum62, -11)
    d = np.argwhere(r.score != S)
    fd = None if len(d) == 0 else (tuple(d[0]), int(r.score[tuple(d[0])]), int(S[tuple(d[0])]), len(d))
    print(f"{R}x{C}: cost {r.align_cost} vs {cost} diff {fd}", flush=True)
    bad += fd is not None
print("BAD", bad)
