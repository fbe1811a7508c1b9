"""Pin the CPU restatement (oracle/) against the reference's own recorded outputs.

The reference is C++/CUDA and cannot be built here (see oracle/nw_oracle.c header), so the
oracle is pinned by the known answers the reference produced, stored in
tests/golden/known_answers.json, on the reference's own input files (tests/golden/resrc).
"""
import numpy as np
import pytest

import oracle


def _hex(v):
    return "%08x" % v


@pytest.mark.parametrize("idx", range(6))
def test_known_answers(golden, idx):
    case = golden.known["cases"][idx]
    Y, X = golden.pair(case["pair"])
    S, cost = oracle.fill_full(Y, X, golden.blosum62, golden.known["gapo"])
    assert cost == case["align_cost"]
    assert _hex(oracle.hash_full(S)) == case["score_hash"]
    th, edit = oracle.trace_full(S, Y, X)
    assert _hex(th) == case["trace_hash"]
    if "edit_trace" in case:
        assert edit == case["edit_trace"]


def test_cpu4_equals_cpu1(golden):
    """cpu4-mt-diagrow restatement == cpu1 (the reference checks this via setOrVerifyResult)."""
    for p, Y, X in golden.pairs("pair_debug.txt")[::11]:
        S1, c1 = oracle.fill_full(Y, X, golden.blosum62, -11)
        for bs in (1, 7, 256):
            S4, c4 = oracle.fill_full_mt(Y, X, golden.blosum62, -11, blocksz=bs, nthreads=4)
            assert c4 == c1 and np.array_equal(S4, S1)


def test_hash_stream_equals_hash1(golden):
    """NwHash2_Sparse's row-streaming recompute == NwHash1_Plain (src/nwtrace2_sparse.cpp:293 quirk)."""
    for p, Y, X in golden.pairs("pair_debug.txt")[::9]:
        S, c = oracle.fill_full(Y, X, golden.blosum62, -11)
        h2, c2 = oracle.hash_stream(Y, X, golden.blosum62, -11)
        assert (h2, c2) == (oracle.hash_full(S), c)


@pytest.mark.parametrize("tBy,tBx", [(32, 54), (252, 256), (63, 64), (7, 3), (128, 209)])
def test_sparse_headers_are_matrix_values(golden, tBy, tBx):
    """Every mlsp header element equals the score-matrix value at its position; Trace2 over the
    headers reproduces Trace1 (the reference compares both families through the same hashes)."""
    for p, Y, X in golden.pairs("pair_debug.txt")[::13]:
        S, cost = oracle.fill_full(Y, X, golden.blosum62, -11)
        hr, hc, tr, tc, c3 = oracle.sparse_headers(Y, X, golden.blosum62, -11, tBy, tBx)
        R, C = len(Y) - 1, len(X) - 1
        hr3, hc3 = hr.reshape(tr, tc, 1 + tBx), hc.reshape(tr, tc, 1 + tBy)
        for iT in range(tr):
            for jT in range(tc):
                i, js = iT * tBy, np.arange(jT * tBx, jT * tBx + tBx + 1)
                m = js <= C
                if i <= R:
                    assert np.array_equal(hr3[iT, jT][m], S[i, js[m]])
                j, is_ = jT * tBx, np.arange(iT * tBy, iT * tBy + tBy + 1)
                m = is_ <= R
                if j <= C:
                    assert np.array_equal(hc3[iT, jT][m], S[is_[m], j])
        th, ed = oracle.trace_full(S, Y, X)
        th2, ed2, c4 = oracle.trace_sparse(hr, hc, tr, tc, tBy, tBx, Y, X, golden.blosum62, -11)
        assert (th2, ed2, c3, c4) == (th, ed, cost, cost)


def test_padding_region_uses_letter_zero():
    """Padded cells (beyond R/C up to the tile multiple) use letter 0, as the reference's
    zero-filled seqX_gpu/seqY_gpu tails do (nwalign_gpu9_mlsp_diagdiagdiag.cu:469-478)."""
    from tests._data import random_pair
    Y, X = random_pair(10, 20, 5)
    sub = np.arange(25 * 25, dtype=np.int32).reshape(25, 25) % 7 - 3
    hr, hc, tr, tc, _ = oracle.sparse_headers(Y, X, sub, -2, 16, 64)
    Yp = np.zeros(1 + tr * 16, np.int32)
    Yp[:len(Y)] = Y
    Xp = np.zeros(1 + tc * 64, np.int32)
    Xp[:len(X)] = X
    S, _ = oracle.fill_full(Yp, Xp, sub, -2)
    assert np.array_equal(hr.reshape(tr, tc, 65)[0, 0], S[0, :65])
    assert np.array_equal(hc.reshape(tr, tc, 17)[0, 0], S[:17, 0])
