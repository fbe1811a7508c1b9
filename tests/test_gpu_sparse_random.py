"""Seeded random shapes over the sparse (mlsp) fill and the device Trace2: lengths 1..4500, tile
widths 64..1024 in steps of 16, related and unrelated pairs, every K-rows geometry the library
ships.  Each fill is compared word for word with the oracle's tile headers
(nwalign_gpu9_mlsp_diagdiagdiag.cu:15-360 as restated in oracle/nw_oracle.c) and each device
trace with the host NwTrace2_Sparse restatement (nwtrace2_sparse.cpp:102-257)."""
import numpy as np
import pytest

import gpuseqalign_amd as gsa
import oracle
from gpuseqalign_amd import formats as F
from tests._data import random_pair

pytestmark = pytest.mark.gpu


def _shapes(seed, n):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        R, C = (int(v) for v in rng.integers(1, 4500, size=2))
        tBx = 64 + 16 * int(rng.integers(0, 61))
        out.append((R, C, tBx, bool(rng.integers(0, 2)), int(rng.integers(0, 1 << 30))))
    return out


def _pair(R, C, related, seed):
    if related:
        X = F.synthetic_seq(C, seed)
        Y = F.mutate_seq(X, seed + 1)[:R + 1]
        return Y, X
    return random_pair(R, C, seed)


@pytest.mark.parametrize("ns,k", [(4, 4), (8, 4), (2, 2)])
def test_random_shapes_match_oracle(engine, golden, monkeypatch, ns, k):
    monkeypatch.setenv("GSA_KROW_NS", str(ns))
    monkeypatch.setenv("GSA_KROW_K", str(k))
    for R, C, tBx, related, seed in _shapes(100 * ns + k, 12):
        Y, X = _pair(R, C, related, seed)
        res = engine.align_sparse(Y, X, golden.blosum62, -11, tileBx=tBx)
        hr, hc, _, _, cost = oracle.sparse_headers(Y, X, golden.blosum62, -11, gsa.sparse_tile_by(), tBx)
        assert np.array_equal(res.hrow, hr) and np.array_equal(res.hcol, hc), (len(Y), len(X), tBx, related)
        assert res.align_cost == cost


def test_random_shapes_device_trace(engine, golden):
    import torch
    dev = torch.device("cuda:0")
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.int32)).to(dev)
    for R, C, tBx, related, seed in _shapes(7, 10):
        Y, X = _pair(R, C, related, seed)
        geom = gsa.sparse_geometry(len(Y), len(X), tBx)
        y, x, s = d(Y), d(X), d(golden.blosum62)
        hr = torch.empty(geom.hrowElems, dtype=torch.int32, device=dev)
        hc = torch.empty(geom.hcolElems, dtype=torch.int32, device=dev)
        args = (y.data_ptr(), len(Y), x.data_ptr(), len(X), s.data_ptr(), 25, -11)
        engine.fill_sparse_dev(*args, tBx, hr.data_ptr(), hc.data_ptr())
        engine.sync()
        got = engine.trace_sparse_dev(*args, geom, hr.data_ptr(), hc.data_ptr())
        res = gsa.SparseResult(hr.cpu().numpy(), hc.cpu().numpy(), geom, 0, {})
        assert got == gsa.trace_sparse(res, Y, X, golden.blosum62, -11), (len(Y), len(X), tBx, related)
