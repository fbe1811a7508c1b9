"""Score-only NW/SW with linear or affine gaps (oracle/score_oracle.c; BASELINE configs[4],
SURVEY.md 8(f)3).  The reference has no implementation of these modes, so the C restatement
is pinned here by (a) the NW-LG special case go == ge == g against orc_fill_full, itself
pinned to the reference's known answers, (b) an independent pure-Python restatement of the
recurrences on small pairs, and (c) the tiled OpenMP wavefront version."""
import numpy as np
import pytest

import oracle
from tests._data import random_pair, related_pair

NEG = -(1 << 29)


def py_score(Y, X, sub, go, ge, local):
    """Gotoh H/E/F, literally (score_oracle.c header)."""
    n = int(round(np.sqrt(np.asarray(sub).size)))
    S = np.asarray(sub).reshape(n, n)
    R, C = len(Y) - 1, len(X) - 1
    hdr = lambda k: 0 if (k == 0 or local) else go + (k - 1) * ge
    H = [[0] * (C + 1) for _ in range(R + 1)]
    E = [[NEG] * (C + 1) for _ in range(R + 1)]
    F = [[NEG] * (C + 1) for _ in range(R + 1)]
    for j in range(C + 1):
        H[0][j] = hdr(j)
    for i in range(R + 1):
        H[i][0] = hdr(i)
    best, bi, bj = 0, 0, 0
    for i in range(1, R + 1):
        for j in range(1, C + 1):
            E[i][j] = max(E[i][j - 1] + ge, H[i][j - 1] + go)
            F[i][j] = max(F[i - 1][j] + ge, H[i - 1][j] + go)
            h = max(H[i - 1][j - 1] + int(S[Y[i], X[j]]), E[i][j], F[i][j])
            if local:
                h = max(h, 0)
            H[i][j] = h
            if local and h > best:
                best, bi, bj = h, i, j
    return (best, bi, bj) if local else (H[R][C], R, C)


@pytest.mark.parametrize("R,C", [(0, 0), (0, 5), (6, 0), (1, 1), (17, 23), (40, 31)])
@pytest.mark.parametrize("go,ge", [(-11, -11), (-11, -1), (-5, -2)])
@pytest.mark.parametrize("local", [False, True])
def test_c_equals_python(golden, R, C, go, ge, local):
    Y, X = random_pair(R, C, 100 * R + C + 7)
    assert oracle.score_ag(Y, X, golden.blosum62, go, ge, local) == py_score(Y, X, golden.blosum62, go, ge, local)


def test_local_on_related_pairs_python(golden):
    Y, X = related_pair(60, 5)
    for go, ge in [(-11, -1), (-8, -8)]:
        assert oracle.score_ag(Y, X, golden.blosum62, go, ge, True) == py_score(Y, X, golden.blosum62, go, ge, True)


def test_linear_global_is_reference_nw_lg(golden):
    """go == ge == g, global: the reference's NW-LG align_cost (orc_fill_full, pinned to known answers)."""
    for _, Y, X in golden.pairs("pair_debug.txt")[:40]:
        _, cost = oracle.fill_full(Y, X, golden.blosum62, -11)
        assert oracle.score_ag(Y, X, golden.blosum62, -11, -11, False)[0] == cost
    for k in golden.known["cases"]:
        if k["pair"].startswith("len12124"):
            continue
        Y, X = golden.pair(k["pair"])
        assert oracle.score_ag(Y, X, golden.blosum62, -11, -11, False)[0] == k["align_cost"]


@pytest.mark.parametrize("R,C,B", [(300, 257, 64), (700, 500, 100), (1000, 1000, 256), (129, 2000, 7)])
@pytest.mark.parametrize("go,ge,local", [(-11, -1, False), (-11, -1, True), (-11, -11, True), (-11, -11, False)])
def test_mt_equals_streaming(golden, R, C, B, go, ge, local):
    Y, X = related_pair(R, R + C) if local else random_pair(R, C, R * C)
    X = X[:C + 1]
    a = oracle.score_ag(Y, X, golden.blosum62, go, ge, local)
    b = oracle.score_ag(Y, X, golden.blosum62, go, ge, local, mt=True, blocksz=B, nthreads=4)
    assert a == b
