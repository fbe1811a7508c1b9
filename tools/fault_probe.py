"""Staged GPU probe for a launch-path change: one small case per call, oracle-checked.
usage: fault_probe.py full|sparse R C   (exit 0 = bit-exact)"""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import gpuseqalign_amd as gsa
import oracle
from tests._data import Golden, random_pair
mode, R, C = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
G = Golden()
Y, X = random_pair(R, C, R * 7 + C)
with gsa.Engine(0) as e:
    if mode == "full":
        r = e.align_full(Y, X, G.blosum62, -11)
        S, cost = oracle.fill_full(Y, X, G.blosum62, -11)
        ok = np.array_equal(r.score, S) and r.align_cost == cost
        d = np.argwhere(r.score != S)
        if len(d):
            print("score ndiff", len(d), "first", [(tuple(int(v) for v in x), int(r.score[tuple(x)]), int(S[tuple(x)])) for x in d[:6]])
    else:
        r = e.align_sparse(Y, X, G.blosum62, -11, tileBx=64)
        hr, hc, _, _, cost = oracle.sparse_headers(Y, X, G.blosum62, -11, gsa.sparse_tile_by(), 64)
        ok = np.array_equal(r.hrow, hr) and np.array_equal(r.hcol, hc) and r.align_cost == cost
        g = r.geom
        for name, a, b, L in (("hrow", r.hrow, hr, g.tileHrowLen), ("hcol", r.hcol, hc, g.tileHcolLen)):
            d = np.nonzero(a != b)[0]
            if len(d):
                t = d // L
                print(name, "ndiff", len(d), "first", [(int(i), int(i // L), int(i % L), int(a[i]), int(b[i])) for i in d[:6]],
                      "tiles", sorted(set((int(x) // g.tileHdrMatCols, int(x) % g.tileHdrMatCols) for x in t))[:12])
print(mode, R, C, "OK" if ok else "MISMATCH", flush=True)
sys.exit(0 if ok else 1)
