"""ctypes bindings for the CPU restatement (nw_oracle.c).

TEST INFRASTRUCTURE ONLY: importable from tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, as the checker.  The product never imports this.
Each wrapper names the reference function it restates (see nw_oracle.c).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

_i32p = ctypes.POINTER(ctypes.c_int32)
_i64 = ctypes.c_int64


def build() -> str:
    """Compile liborc.so (gcc) if missing or stale."""
    so = os.path.join(_HERE, "liborc.so")
    srcs = [os.path.join(_HERE, f) for f in ("nw_oracle.c", "score_oracle.c", "Makefile")]
    if not os.path.exists(so) or os.path.getmtime(so) < max(os.path.getmtime(f) for f in srcs):
        subprocess.check_call(["make", "-s", "-C", _HERE])
    return so


def lib():
    global _LIB
    if _LIB is None:
        so = build()
        L = ctypes.CDLL(so)
        L.orc_fill_full.restype = ctypes.c_int32
        L.orc_fill_full.argtypes = [_i32p, _i64, _i32p, _i64, _i32p, ctypes.c_int32, ctypes.c_int32, _i32p]
        L.orc_fill_full_mt.restype = ctypes.c_int32
        L.orc_fill_full_mt.argtypes = [_i32p, _i64, _i32p, _i64, _i32p, ctypes.c_int32, ctypes.c_int32, _i32p,
                                       ctypes.c_int32, ctypes.c_int32]
        L.orc_hash_full.restype = ctypes.c_uint32
        L.orc_hash_full.argtypes = [_i32p, _i64, _i64]
        L.orc_trace_full.restype = ctypes.c_uint32
        L.orc_trace_full.argtypes = [_i32p, _i32p, _i64, _i32p, _i64, ctypes.c_char_p, _i64,
                                     ctypes.POINTER(ctypes.c_int64)]
        L.orc_sparse_headers.restype = ctypes.c_int32
        L.orc_sparse_headers.argtypes = [_i32p, _i64, _i32p, _i64, _i32p, ctypes.c_int32, ctypes.c_int32,
                                         ctypes.c_int32, ctypes.c_int32, _i32p, _i32p]
        L.orc_hash_stream.restype = ctypes.c_uint32
        L.orc_hash_stream.argtypes = [_i32p, _i64, _i32p, _i64, _i32p, ctypes.c_int32, ctypes.c_int32, _i32p]
        L.orc_trace_sparse.restype = ctypes.c_uint32
        L.orc_trace_sparse.argtypes = [_i32p, _i32p, _i64, _i64, _i64, _i64, _i32p, _i64, _i32p, _i64, _i32p,
                                       ctypes.c_int32, ctypes.c_int32, ctypes.c_char_p, _i64,
                                       ctypes.POINTER(ctypes.c_int64), _i32p]
        L.orc_score_ag.restype = ctypes.c_int32
        L.orc_score_ag.argtypes = [_i32p, _i64, _i32p, _i64, _i32p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                   ctypes.c_int32, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]
        L.orc_score_ag_mt.restype = ctypes.c_int32
        L.orc_score_ag_mt.argtypes = [_i32p, _i64, _i32p, _i64, _i32p, ctypes.c_int32, ctypes.c_int32,
                                      ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                      ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]
        _LIB = L
    return _LIB


def _p(a: np.ndarray):
    assert a.dtype == np.int32 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(_i32p)


def fill_full(seqY, seqX, subst, g):
    """NwAlign_Cpu1_St_Row (src/nwalign_cpu1_st_row.cpp:12-67) -> (score[adjrows, adjcols], align_cost)."""
    seqY = np.ascontiguousarray(seqY, np.int32)
    seqX = np.ascontiguousarray(seqX, np.int32)
    subst = np.ascontiguousarray(subst, np.int32)
    substsz = int(round(np.sqrt(subst.size)))
    score = np.empty((len(seqY), len(seqX)), dtype=np.int32)
    cost = lib().orc_fill_full(_p(seqY), len(seqY), _p(seqX), len(seqX), _p(subst), substsz, g, _p(score))
    return score, int(cost)


def fill_full_mt(seqY, seqX, subst, g, blocksz=256, nthreads=0):
    """NwAlign_Cpu4_Mt_DiagRow (src/nwalign_cpu4_mt_diagrow.cpp:13-111)."""
    seqY = np.ascontiguousarray(seqY, np.int32)
    seqX = np.ascontiguousarray(seqX, np.int32)
    subst = np.ascontiguousarray(subst, np.int32)
    substsz = int(round(np.sqrt(subst.size)))
    score = np.empty((len(seqY), len(seqX)), dtype=np.int32)
    cost = lib().orc_fill_full_mt(_p(seqY), len(seqY), _p(seqX), len(seqX), _p(subst), substsz, g, _p(score),
                                  blocksz, nthreads)
    return score, int(cost)


def hash_full(score: np.ndarray) -> int:
    """NwHash1_Plain (src/nwtrace1_plain.cpp:133-154)."""
    score = np.ascontiguousarray(score, np.int32)
    return int(lib().orc_hash_full(_p(score), score.shape[0], score.shape[1]))


def trace_full(score, seqY, seqX):
    """NwTrace1_Plain (src/nwtrace1_plain.cpp:6-131) -> (trace_hash, edit_trace)."""
    score = np.ascontiguousarray(score, np.int32)
    seqY = np.ascontiguousarray(seqY, np.int32)
    seqX = np.ascontiguousarray(seqX, np.int32)
    cap = 2 * (len(seqY) + len(seqX)) * 8 + 64
    buf = ctypes.create_string_buffer(cap)
    n = ctypes.c_int64(0)
    h = lib().orc_trace_full(_p(score), _p(seqY), len(seqY), _p(seqX), len(seqX), buf, cap, ctypes.byref(n))
    assert n.value >= 0
    return int(h), buf.raw[:n.value].decode()


def sparse_geometry(adjrows, adjcols, tBy, tBx):
    trows = max(1, (adjrows - 1 + tBy - 1) // tBy)
    tcols = max(1, (adjcols - 1 + tBx - 1) // tBx)
    return trows, tcols


def sparse_headers(seqY, seqX, subst, g, tBy, tBx):
    """mlsp tile headers as gpu7-9 leave them (nwalign_gpu9_mlsp_diagdiagdiag.cu:15-360).

    Returns (hrow[trows*tcols*(1+tBx)], hcol[trows*tcols*(1+tBy)], trows, tcols, align_cost)."""
    seqY = np.ascontiguousarray(seqY, np.int32)
    seqX = np.ascontiguousarray(seqX, np.int32)
    subst = np.ascontiguousarray(subst, np.int32)
    substsz = int(round(np.sqrt(subst.size)))
    trows, tcols = sparse_geometry(len(seqY), len(seqX), tBy, tBx)
    hrow = np.empty(trows * tcols * (1 + tBx), dtype=np.int32)
    hcol = np.empty(trows * tcols * (1 + tBy), dtype=np.int32)
    cost = lib().orc_sparse_headers(_p(seqY), len(seqY), _p(seqX), len(seqX), _p(subst), substsz, g, tBy, tBx,
                                    _p(hrow), _p(hcol))
    return hrow, hcol, trows, tcols, int(cost)


def hash_stream(seqY, seqX, subst, g):
    """NwHash2_Sparse as it behaves (== NwHash1_Plain, src/nwtrace2_sparse.cpp:263-340) -> (hash, cost)."""
    seqY = np.ascontiguousarray(seqY, np.int32)
    seqX = np.ascontiguousarray(seqX, np.int32)
    subst = np.ascontiguousarray(subst, np.int32)
    substsz = int(round(np.sqrt(subst.size)))
    cost = np.zeros(1, dtype=np.int32)
    h = lib().orc_hash_stream(_p(seqY), len(seqY), _p(seqX), len(seqX), _p(subst), substsz, g, _p(cost))
    return int(h), int(cost[0])


def trace_sparse(hrow, hcol, trows, tcols, tBy, tBx, seqY, seqX, subst, g):
    """NwTrace2_Sparse (src/nwtrace2_sparse.cpp:102-257) -> (trace_hash, edit_trace, align_cost)."""
    hrow = np.ascontiguousarray(hrow, np.int32)
    hcol = np.ascontiguousarray(hcol, np.int32)
    seqY = np.ascontiguousarray(seqY, np.int32)
    seqX = np.ascontiguousarray(seqX, np.int32)
    subst = np.ascontiguousarray(subst, np.int32)
    substsz = int(round(np.sqrt(subst.size)))
    cap = 2 * (len(seqY) + len(seqX)) * 8 + 64
    buf = ctypes.create_string_buffer(cap)
    n = ctypes.c_int64(0)
    cost = np.zeros(1, dtype=np.int32)
    h = lib().orc_trace_sparse(_p(hrow), _p(hcol), trows, tcols, 1 + tBx, 1 + tBy, _p(seqY), len(seqY), _p(seqX),
                               len(seqX), _p(subst), substsz, g, buf, cap, ctypes.byref(n), _p(cost))
    assert n.value >= 0
    return int(h), buf.raw[:n.value].decode(), int(cost[0])


def score_ag(seqY, seqX, subst, go: int, ge: int, local: bool = False, mt: bool = False, blocksz: int = 256,
             nthreads: int = 0):
    """Score-only NW / SW with affine gaps (score_oracle.c; linear gaps: go == ge).
    Returns (score, i_end, j_end).  Not in the reference: parity unpinned by it (see the C header)."""
    y, x, s = (np.ascontiguousarray(a, dtype=np.int32) for a in (seqY, seqX, subst))
    substsz = int(round(np.sqrt(s.size)))
    ie, je = ctypes.c_int64(0), ctypes.c_int64(0)
    if mt:
        sc = lib().orc_score_ag_mt(_p(y), len(y), _p(x), len(x), _p(s.ravel()), substsz, go, ge, int(local), blocksz,
                                   nthreads, ctypes.byref(ie), ctypes.byref(je))
    else:
        sc = lib().orc_score_ag(_p(y), len(y), _p(x), len(x), _p(s.ravel()), substsz, go, ge, int(local),
                                ctypes.byref(ie), ctypes.byref(je))
    return int(sc), int(ie.value), int(je.value)
