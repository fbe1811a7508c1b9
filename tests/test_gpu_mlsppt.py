"""mlsppt -- sparse fill with the header copy-back overlapped with the fill (gsa_align_sparse_pt;
named in the reference's README.md:39, never implemented there): every word
of both header matrices, the geometry and align_cost equal the plain mlsp path's."""
import numpy as np
import pytest

from tests._data import random_pair, related_pair

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("R,C,tBx", [(1, 1, 64), (700, 900, 64), (5000, 3000, 256), (20000, 9000, 512),
                                     (40000, 40000, 256)])
def test_overlap_equals_plain(engine, golden, R, C, tBx):
    Y, X = related_pair(R, R + 1) if R == C else random_pair(R, C, R + C)
    a = engine.align_sparse(Y, X, golden.blosum62, -11, tileBx=tBx)
    for _ in range(2):  # the per-ticket flags of the previous launch must not count as done
        b = engine.align_sparse(Y, X, golden.blosum62, -11, tileBx=tBx, overlap=True)
        assert np.array_equal(a.hrow, b.hrow) and np.array_equal(a.hcol, b.hcol)
        assert a.align_cost == b.align_cost
        assert (a.geom.tileHdrMatRows, a.geom.tileHdrMatCols) == (b.geom.tileHdrMatRows, b.geom.tileHdrMatCols)


@pytest.mark.parametrize("kern,ns,k", [("krow", 2, 2), ("krow", 8, 4), ("strip", 4, 4)])
def test_overlap_other_geometries(engine, golden, monkeypatch, kern, ns, k):
    """mlsppt flags one ticket per tile row: a K-rows geometry whose ticket is not one tile row
    (GSA_KROW_NS / GSA_KROW_K) falls back to the single-pair default, and the strip kernel
    (GSA_SPARSE_KERNEL=strip) flags its own tickets; every word equals the plain path's."""
    import oracle
    Y, X = random_pair(3100, 2200, 41)
    a = engine.align_sparse(Y, X, golden.blosum62, -11, tileBx=128)
    monkeypatch.setenv("GSA_SPARSE_KERNEL", kern)
    monkeypatch.setenv("GSA_KROW_NS", str(ns))
    monkeypatch.setenv("GSA_KROW_K", str(k))
    b = engine.align_sparse(Y, X, golden.blosum62, -11, tileBx=128, overlap=True)
    assert np.array_equal(a.hrow, b.hrow) and np.array_equal(a.hcol, b.hcol)
    assert a.align_cost == b.align_cost == oracle.fill_full(Y, X, golden.blosum62, -11)[1]
