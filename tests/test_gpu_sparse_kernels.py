"""Every sparse-fill kernel the library ships, word for word against the oracle's tile headers
(nwalign_gpu9_mlsp_diagdiagdiag.cu:15-360 as restated in oracle/nw_oracle.c): the K-rows kernel
(nw_krow.hip) in each geometry it instantiates and the strip kernel (nw_strip.hip, which mlsppt and
GSA_SPARSE_KERNEL=strip use).  The kernel choice is read from the environment per launch."""
import numpy as np
import pytest

import gpuseqalign_amd as gsa
import oracle
from tests._data import random_pair, related_pair

pytestmark = pytest.mark.gpu

# (kernel, strips per workgroup, rows per lane)
KERNELS = [("krow", 4, 4), ("krow", 8, 4), ("krow", 4, 2), ("krow", 2, 4), ("krow", 2, 2), ("strip", 4, 4)]


def _select(monkeypatch, kern, ns, k):
    monkeypatch.setenv("GSA_SPARSE_KERNEL", kern)
    monkeypatch.setenv("GSA_KROW_NS", str(ns))
    monkeypatch.setenv("GSA_KROW_K", str(k))


@pytest.mark.parametrize("kern,ns,k", KERNELS)
@pytest.mark.parametrize("R,C,tBx,related", [(1, 1, 64, False), (63, 2000, 64, False), (1500, 700, 80, True),
                                             (2049, 3001, 256, True), (4100, 1030, 512, False),
                                             (700, 1900, 96, True), (1100, 1777, 112, False), (3000, 2500, 128, True),
                                             (130, 5000, 64, True)])
def test_sparse_kernel_matches_oracle(engine, golden, monkeypatch, kern, ns, k, R, C, tBx, related):
    _select(monkeypatch, kern, ns, k)
    Y, X = related_pair(max(R, C), 31) if related else random_pair(R, C, 17)
    Y, X = Y[:R + 1], X[:C + 1]
    res = engine.align_sparse(Y, X, golden.blosum62, -11, tileBx=tBx)
    hr, hc, _, _, cost = oracle.sparse_headers(Y, X, golden.blosum62, -11, gsa.sparse_tile_by(), tBx)
    assert np.array_equal(res.hrow, hr) and np.array_equal(res.hcol, hc)
    assert res.align_cost == cost


@pytest.mark.parametrize("kern,ns,k", KERNELS)
def test_sparse_kernel_batch_matches_oracle(golden, monkeypatch, kern, ns, k):
    """A batched launch (tickets of several pairs interleaved) in each geometry."""
    import torch
    from gpuseqalign_amd import shard
    _select(monkeypatch, kern, ns, k)
    if not torch.cuda.is_available():
        pytest.skip("no GPU visible")
    pairs = shard.synthetic_batch(12, 300, 2600, seed0=77)
    costs, _ = shard.gpu_batch_align(0, mode="sparse", tileBx=128)(list(range(len(pairs))), pairs, golden.blosum62, -11)
    for (y, x), c in zip(pairs, costs):
        assert c == oracle.fill_full(y, x, golden.blosum62, -11)[1]


def test_sparse_profile_range_is_checked(engine, golden):
    """The K-rows kernel keeps s - 2g in int16: a gap cost that breaks it fails loudly."""
    Y, X = random_pair(300, 400, 3)
    with pytest.raises(gsa.NwError):
        engine.align_sparse(Y, X, golden.blosum62, -20000, tileBx=64)
    # the context is usable afterwards
    res = engine.align_sparse(Y, X, golden.blosum62, -11, tileBx=64)
    assert res.align_cost == oracle.fill_full(Y, X, golden.blosum62, -11)[1]


@pytest.mark.parametrize("R,C", [(63, 2000), (1500, 1300), (3000, 2100)])
@pytest.mark.parametrize("gapo,q8", [(-11, "0"), (-80, "1"), (-59, "1"), (-58, "1"), (-11, "1")])
def test_krow_profile_width(engine, golden, R, C, gapo, q8, monkeypatch, knobs):
    """The K-rows fill keeps s - 2g in an int8 column profile when the table allows it and falls
    back to the int16 instance otherwise (blosum62 has -4 <= s <= 11: gapo -58 fits, s + 116 <= 127;
    -59 and -80 do not, and their int8 launches decline; a fitting fill after a declined one checks
    that the per-launch word is not stale); GSA_KROW_Q8=0 forces int16.  Headers word for word
    against the oracle."""
    import oracle
    knobs("GSA_SPARSE_KERNEL", None)
    monkeypatch.setenv("GSA_KROW_Q8", q8)
    Y, X = random_pair(R, C, R + 3 * C)
    res = engine.align_sparse(Y, X, golden.blosum62, gapo, tileBx=256)
    hr, hc, _, _, cost = oracle.sparse_headers(Y, X, golden.blosum62, gapo, gsa.sparse_tile_by(), 256)
    assert np.array_equal(res.hrow, hr) and np.array_equal(res.hcol, hc)
    assert res.align_cost == cost


@pytest.mark.parametrize("kern,ns,k", KERNELS)
def test_sparse_kernel_batch_declined_table(golden, monkeypatch, kern, ns, k):
    """A batch whose table leaves int8 (gapo -80): every geometry's int8 instance declines and the
    int16 instance behind it fills the batch."""
    import torch
    from gpuseqalign_amd import shard
    _select(monkeypatch, kern, ns, k)
    if not torch.cuda.is_available():
        pytest.skip("no GPU visible")
    pairs = shard.synthetic_batch(12, 300, 2600, seed0=91)
    costs, _ = shard.gpu_batch_align(0, mode="sparse", tileBx=128)(list(range(len(pairs))), pairs, golden.blosum62, -80)
    for (y, x), c in zip(pairs, costs):
        assert c == oracle.fill_full(y, x, golden.blosum62, -80)[1]


@pytest.mark.parametrize("gapo", [-80, -11])
def test_overlap_declined_table(engine, golden, gapo):
    """mlsppt (the PT instances) with a table outside int8 and then inside it, headers against the
    oracle."""
    Y, X = random_pair(3000, 9000, 5)
    hr, hc, _, _, cost = oracle.sparse_headers(Y, X, golden.blosum62, gapo, gsa.sparse_tile_by(), 256)
    b = engine.align_sparse(Y, X, golden.blosum62, gapo, tileBx=256, overlap=True)
    assert np.array_equal(b.hrow, hr) and np.array_equal(b.hcol, hc)
    assert b.align_cost == cost
