"""The C-ABI library: loads, exports every symbol include/gsa.h declares, and its host-side
consumers (Trace1/Hash1/Trace2/Hash2, src/nwtrace1_plain.cpp / src/nwtrace2_sparse.cpp)
agree with the oracle.  No GPU compute here."""
import os
import re

import numpy as np
import pytest

import gpuseqalign_amd as gsa
import oracle
from tests._data import random_pair

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    text = open(os.path.join(ROOT, "include", "gsa.h")).read()
    return sorted(set(re.findall(r"\b(gsa_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_header():
    L = gsa.lib()
    decl = declared_symbols()
    assert len(decl) >= 15
    for name in decl:
        assert hasattr(L, name), name
        assert name in gsa.SIGNATURES, name


def test_geometry():
    g = gsa.sparse_geometry(10001, 10001, 256)
    assert g.tileBy == gsa.sparse_tile_by() == 1024
    assert g.tileHdrMatRows == -(-10000 // 1024) and g.tileHdrMatCols == -(-10000 // 256)
    assert g.hrowElems == g.tileHdrMatRows * g.tileHdrMatCols * 257
    e = gsa.sparse_geometry(1, 1, 64)  # empty sequences -> one tile (gpu9 host :419-426)
    assert (e.tileHdrMatRows, e.tileHdrMatCols) == (1, 1)
    with pytest.raises(gsa.NwError):
        gsa.sparse_geometry(10, 10, 50)


def test_host_trace_hash_match_oracle(golden):
    for p, Y, X in golden.pairs("pair_debug.txt")[::5]:
        S, _ = oracle.fill_full(Y, X, golden.blosum62, -11)
        assert gsa.hash_full(S) == oracle.hash_full(S)
        assert gsa.trace_full(S, Y, X) == oracle.trace_full(S, Y, X)


@pytest.mark.parametrize("tBx", [64, 256])
def test_host_sparse_consumers_match_oracle(golden, tBx):
    tBy = gsa.sparse_tile_by()
    cases = [golden.pair("len64 len728"), golden.pair("len728 len728"), random_pair(600, 333, 7),
             golden.pair("len1 len1")]
    for Y, X in cases:
        hr, hc, tr, tc, cost = oracle.sparse_headers(Y, X, golden.blosum62, -11, tBy, tBx)
        geom = gsa.sparse_geometry(len(Y), len(X), tBx)
        assert (geom.tileHdrMatRows, geom.tileHdrMatCols) == (tr, tc)
        res = gsa.SparseResult(hr, hc, geom, cost, {})
        th, ed, c = gsa.trace_sparse(res, Y, X, golden.blosum62, -11)
        oth, oed, oc = oracle.trace_sparse(hr, hc, tr, tc, tBy, tBx, Y, X, golden.blosum62, -11)
        assert (th, ed, c) == (oth, oed, oc)
        assert gsa.sparse_align_cost(res, Y, X, golden.blosum62, -11) == cost
        assert gsa.hash_sparse(res, Y, X, golden.blosum62, -11) == oracle.hash_stream(Y, X, golden.blosum62, -11)[0]


def test_registry_names():
    m = gsa.get_nw_algorithm_map()
    assert m["NwAlign_Gpu9_Mlsp_DiagDiagDiag"].trace is m["NwAlign_Amd_Strip_Mlsp"].trace
    assert m["NwAlign_Gpu3_Ml_DiagDiag"].hash is m["NwAlign_Amd_Strip_Full"].hash
