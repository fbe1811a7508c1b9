"""Device-side verification (gsa_check_sparse_dev / gsa_check_full_dev, nw_check.hip;
SURVEY.md 8(f)1).

The checker is first pinned on outputs it did not produce: the oracle's headers and
matrices (CPU restatement of the reference's cpu1-st-row + mlsp header extraction) must
check clean, and single corrupted values must be caught.  It then checks the HIP fills,
including full-size sparse fills (100k x 100k, BASELINE configs[2]) that no CPU oracle
run fits into a test: zero mismatches over every header value is the size-independent
parity property at that size.
"""
import numpy as np
import pytest

import gpuseqalign_amd as gsa
from tests._data import random_pair, related_pair

pytestmark = pytest.mark.gpu


def _dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.int32)).to("cuda:0")


def _expected_sparse_checks(geom):
    tr, tc, W, H = geom.tileHdrMatRows, geom.tileHdrMatCols, geom.tileHrowLen, geom.tileHcolLen
    return tr * H + tc * W + tr * tc + (tr - 1) * tc * W + tr * (tc - 1) * H


def _check_sparse(engine, Y, X, sub, gapo, geom, hr, hc):
    y, x, s = _dev(Y), _dev(X), _dev(sub)
    return engine.check_sparse_dev(y.data_ptr(), len(Y), x.data_ptr(), len(X), s.data_ptr(), int(round(np.sqrt(sub.size))), gapo,
                                   geom, hr.data_ptr(), hc.data_ptr())


def _fill_sparse(engine, Y, X, sub, gapo, tBx):
    import torch
    geom = gsa.sparse_geometry(len(Y), len(X), tBx)
    y, x, s = _dev(Y), _dev(X), _dev(sub)
    hr = torch.full((geom.hrowElems,), -7, dtype=torch.int32, device="cuda:0")
    hc = torch.full((geom.hcolElems,), -7, dtype=torch.int32, device="cuda:0")
    engine.fill_sparse_dev(y.data_ptr(), len(Y), x.data_ptr(), len(X), s.data_ptr(), int(round(np.sqrt(sub.size))), gapo, tBx,
                           hr.data_ptr(), hc.data_ptr())
    engine.sync()
    return geom, hr, hc


@pytest.mark.parametrize("R,C,tBx", [(1, 1, 64), (700, 900, 64), (1100, 3000, 80), (2049, 1000, 256),
                                     (3000, 257, 512)])
def test_checker_on_oracle_headers(engine, golden, R, C, tBx):
    import oracle
    Y, X = random_pair(R, C, 11 * R + C)
    geom = gsa.sparse_geometry(len(Y), len(X), tBx)
    hr, hc, _, _, _ = oracle.sparse_headers(Y, X, golden.blosum62, -11, geom.tileBy, tBx)
    r = _check_sparse(engine, Y, X, golden.blosum62, -11, geom, _dev(hr), _dev(hc))
    assert r["mismatches"] == 0 and r["first"] == -1, r
    assert r["checked"] == _expected_sparse_checks(geom)


def test_checker_catches_corruption(engine, golden):
    import oracle
    Y, X = related_pair(2500, 21)
    geom = gsa.sparse_geometry(len(Y), len(X), 128)
    hr, hc, _, _, _ = oracle.sparse_headers(Y, X, golden.blosum62, -11, geom.tileBy, 128)
    rng = np.random.default_rng(3)
    W, H, tc = geom.tileHrowLen, geom.tileHcolLen, geom.tileHdrMatCols
    # row 0 of tile (0, 2): a boundary value, reported exactly
    bad = hr.copy()
    bad[2 * W + 5] += 1
    r = _check_sparse(engine, Y, X, golden.blosum62, -11, geom, _dev(bad), _dev(hc))
    assert r["mismatches"] >= 1 and r["first"] == 2 * W + 5, r
    # interior header row / column values, anywhere in the padded matrix
    for _ in range(6):
        which = rng.integers(2)
        b_hr, b_hc = hr.copy(), hc.copy()
        if which == 0:
            k = int(rng.integers(tc, geom.hrowElems // W)) * W + int(rng.integers(1, W))  # tile row >= 1
            b_hr[k] -= int(rng.integers(1, 5))
        else:
            t = int(rng.integers(0, geom.hcolElems // H))
            if t % tc == 0:
                t += 1  # tile column >= 1
            k = t * H + int(rng.integers(1, H))
            b_hc[k] += int(rng.integers(1, 5))
        r = _check_sparse(engine, Y, X, golden.blosum62, -11, geom, _dev(b_hr), _dev(b_hc))
        assert r["mismatches"] >= 1, (which, k, r)


@pytest.mark.parametrize("R,C,tBx", [(700, 900, 64), (1023, 1025, 80), (5000, 4000, 256), (2500, 9000, 512),
                                     (9000, 2000, 4096)])
def test_fill_sparse_checks_clean(engine, golden, R, C, tBx):
    Y, X = related_pair(R, 7 * R) if R == C else random_pair(R, C, R + 3 * C)
    geom, hr, hc = _fill_sparse(engine, Y, X, golden.blosum62, -11, tBx)
    r = _check_sparse(engine, Y, X, golden.blosum62, -11, geom, hr, hc)
    assert r["mismatches"] == 0, r
    assert r["checked"] == _expected_sparse_checks(geom)


def test_full_checker(engine, golden):
    import oracle
    import torch
    Y, X = random_pair(1500, 1300, 77)
    S, _ = oracle.fill_full(Y, X, golden.blosum62, -11)
    y, x, s = _dev(Y), _dev(X), _dev(golden.blosum62)
    args = (y.data_ptr(), len(Y), x.data_ptr(), len(X), s.data_ptr(), 25, -11)
    d = _dev(S.ravel())
    r = engine.check_full_dev(*args, d.data_ptr())
    assert r == {"checked": S.size, "mismatches": 0, "first": -1}
    d[123 * len(X) + 456] += 2
    r = engine.check_full_dev(*args, d.data_ptr())
    assert r["mismatches"] >= 1 and r["first"] == 123 * len(X) + 456
    # the HIP full fill of the same pair
    out = torch.full((S.size,), -7, dtype=torch.int32, device="cuda:0")
    engine.fill_full_dev(*args, out.data_ptr())
    engine.sync()
    assert engine.check_full_dev(*args, out.data_ptr())["mismatches"] == 0


def test_10k_full_checks_clean(engine, golden):
    """BASELINE configs[1] pair: the HIP full fill, every cell checked on the device."""
    import torch
    Y, X = golden.pair("len12124[:10000] len15390[:10000]")
    y, x, s = _dev(Y), _dev(X), _dev(golden.blosum62)
    args = (y.data_ptr(), len(Y), x.data_ptr(), len(X), s.data_ptr(), 25, -11)
    out = torch.empty(len(Y) * len(X), dtype=torch.int32, device="cuda:0")
    engine.fill_full_dev(*args, out.data_ptr())
    engine.sync()
    r = engine.check_full_dev(*args, out.data_ptr())
    assert r["mismatches"] == 0 and r["checked"] == len(Y) * len(X)


@pytest.mark.parametrize("n,tBx", [(100000, 256)])
def test_100k_sparse_checks_clean(engine, golden, n, tBx):
    """BASELINE configs[2]: 100k x 100k sparse fill (related pair, SURVEY.md 8d seeds 100/101),
    every one of its ~84M header values checked against the recurrence on the device."""
    from gpuseqalign_amd import formats as F
    X = F.synthetic_seq(n, 100)
    Y = F.mutate_seq(X, 101)
    geom, hr, hc = _fill_sparse(engine, Y, X, golden.blosum62, -11, tBx)
    r = _check_sparse(engine, Y, X, golden.blosum62, -11, geom, hr, hc)
    assert r["mismatches"] == 0, r
    assert r["checked"] == _expected_sparse_checks(geom)
