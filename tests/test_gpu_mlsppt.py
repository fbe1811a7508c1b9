"""mlsppt -- sparse fill with the header copy-back overlapped with the fill (gsa_align_sparse_pt;
named in the reference's README.md:39, never implemented there): the kernel
publishes column chunks of the headers (every tile row's header rows and columns of ~4096 columns)
as they become final, and the host copies each while the fill runs.  Every word of both header
matrices and align_cost equal the oracle's (tests below) and the plain mlsp path's."""
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


@pytest.mark.parametrize("R,C,tBx", [(1, 1, 64), (700, 900, 64), (3000, 20000, 64), (5000, 3000, 256),
                                     (9000, 33000, 512), (2100, 70000, 4096)])
def test_overlap_equals_oracle(engine, golden, R, C, tBx):
    """Every header word against the oracle's streaming extractor, on shapes of one to many
    column chunks (the last chunk partial) and one to several tile rows, run twice (the words
    of the previous launch carry an older epoch and must not count)."""
    import oracle
    import gpuseqalign_amd as gsa
    Y, X = random_pair(R, C, 3 * R + C)
    hr, hc, tr, tc, cost = oracle.sparse_headers(Y, X, golden.blosum62, -11, gsa.sparse_tile_by(), tBx)
    for _ in range(2):
        b = engine.align_sparse(Y, X, golden.blosum62, -11, tileBx=tBx, overlap=True)
        assert (b.geom.tileHdrMatRows, b.geom.tileHdrMatCols) == (tr, tc)
        assert np.array_equal(b.hrow, hr) and np.array_equal(b.hcol, hc)
        assert b.align_cost == cost


@pytest.mark.parametrize("kern,ns,k", [("krow", 2, 2), ("krow", 8, 4), ("strip", 4, 4)])
def test_overlap_other_geometries(engine, golden, monkeypatch, kern, ns, k, knobs):
    """mlsppt publishes one word per tile row from the K-rows kernel: a geometry whose ticket is
    not one tile row (GSA_KROW_NS / GSA_KROW_K), or GSA_SPARSE_KERNEL=strip, falls back to the
    single-pair default geometry; every word equals the plain path's."""
    import oracle
    Y, X = random_pair(3100, 2200, 41)
    a = engine.align_sparse(Y, X, golden.blosum62, -11, tileBx=128)
    knobs("GSA_SPARSE_KERNEL", kern)
    knobs("GSA_KROW_NS", str(ns))
    knobs("GSA_KROW_K", str(k))
    b = engine.align_sparse(Y, X, golden.blosum62, -11, tileBx=128, overlap=True)
    assert np.array_equal(a.hrow, b.hrow) and np.array_equal(a.hcol, b.hcol)
    assert a.align_cost == b.align_cost == oracle.fill_full(Y, X, golden.blosum62, -11)[1]


def test_overlap_error_then_recovers(golden):
    """A fill that fails while its chunks are being copied (watchdog 0: every wait gives up at once)
    makes mlsppt report errorKernelFailure, with the copies it had issued drained before it
    returns; the next mlsppt call on the same context is exact."""
    import gpuseqalign_amd as gsa
    import oracle
    Y, X = related_pair(20000, 7)
    sub = golden.blosum62
    with gsa.Engine(0) as eng:
        eng.set_watchdog(0)
        with pytest.raises(gsa.NwError) as ei:
            eng.align_sparse(Y, X, sub, -11, tileBx=256, overlap=True)
        assert ei.value.stat == gsa.NwStat.errorKernelFailure
        eng.set_watchdog(1000000)
        r = eng.align_sparse(Y, X, sub, -11, tileBx=256, overlap=True)
    hr, hc, _, _, cost = oracle.sparse_headers(Y, X, sub, -11, gsa.sparse_tile_by(), 256)
    assert np.array_equal(r.hrow, hr) and np.array_equal(r.hcol, hc) and r.align_cost == cost


def test_overlap_tall_pair_narrow_chunks(engine, golden):
    """A tall pair at tBx 64: two 4096-column chunks of every tile row would need
    ~150 MB of pinned staging, so the chunk width shrinks until two chunks fit the 64 MB slots;
    the headers still equal the plain mlsp path's word for word."""
    Y, X = random_pair(140000, 5000, 77)
    a = engine.align_sparse(Y, X, golden.blosum62, -11, tileBx=64)
    b = engine.align_sparse(Y, X, golden.blosum62, -11, tileBx=64, overlap=True)
    assert np.array_equal(a.hrow, b.hrow) and np.array_equal(a.hcol, b.hcol)
    assert a.align_cost == b.align_cost
