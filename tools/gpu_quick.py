"""Quick GPU probe: run a ladder of shapes through libgsa and print the first mismatch
against the oracle (diagnostics for gpurun sessions)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import gpuseqalign_amd as gsa
import oracle
from tests._data import Golden, random_pair

def first_diff(a, b):
    d = np.argwhere(a != b)
    return None if len(d) == 0 else (tuple(d[0]), int(a[tuple(d[0])]), int(b[tuple(d[0])]), len(d))

def main():
    G = Golden()
    eng = gsa.Engine(0)
    print("cu_count", eng.cu_count, flush=True)
    shapes = [(1, 1), (5, 7), (63, 64), (64, 64), (200, 300), (256, 256), (257, 300), (600, 1000), (1023, 500), (1025, 1029), (2000, 1500), (3100, 2222)]
    bad = 0
    for R, C in shapes:
        Y, X = random_pair(R, C, R * 31 + C)
        t = time.time()
        r = eng.align_full(Y, X, G.blosum62, -11)
        S, cost = oracle.fill_full(Y, X, G.blosum62, -11)
        fd = first_diff(r.score, S)
        print(f"full {R}x{C}: cost {r.align_cost} vs {cost} diff {fd} laps {r.laps} {time.time()-t:.3f}s", flush=True)
        bad += fd is not None
        rs = eng.align_sparse(Y, X, G.blosum62, -11, tileBx=64)
        hr, hc, tr, tc, c2 = oracle.sparse_headers(Y, X, G.blosum62, -11, gsa.sparse_tile_by(), 64)
        fr = first_diff(rs.hrow, hr); fc = first_diff(rs.hcol, hc)
        print(f"  mlsp: cost {rs.align_cost} vs {c2} hrow {fr} hcol {fc}", flush=True)
        bad += (fr is not None) + (fc is not None)
    print("BAD", bad)
    return 1 if bad else 0

if __name__ == "__main__":
    sys.exit(main())
