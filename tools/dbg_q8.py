import os, sys
sys.path.insert(0, os.getcwd())
import numpy as np
import gpuseqalign_amd as gsa, oracle
from tests._data import random_pair
from tests._data import Golden
from gpuseqalign_amd import formats as F
sub = F.read_subst_json("tests/golden/resrc/subst.json").matrix("blosum62")
eng = gsa.Engine(0)
R, C = 63, 2000
Y, X = random_pair(R, C, R + 3 * C)
hr, hc, _, _, cost = oracle.sparse_headers(Y, X, sub, -11, gsa.sparse_tile_by(), 256)
for q8 in ("0", "1"):
    os.environ["GSA_KROW_Q8"] = q8
    res = eng.align_sparse(Y, X, sub, -11, tileBx=256)
    bad = np.nonzero(res.hcol != hc)[0]
    print("q8", q8, "cost", res.align_cost, cost, "hrow ok", np.array_equal(res.hrow, hr), "hcol bad", len(bad), bad[:10], bad[-5:] if len(bad) else None)
    if len(bad):
        i = bad[0]
        print("  got", res.hcol[i:i+6], "want", hc[i:i+6], "tile", i // 1025, "elem", i % 1025)
