"""gpuseqalign_amd -- MI355X-native NW-LG engine (drop-in for GpuSeqAlign's align path).

Python host side over the C ABI of ``libgsa.so`` (include/gsa.h).  The compute path is the
hand-written gfx950 HIP kernels in ``csrc/`` (``nw_krow.hip`` sparse fills, ``nw_lane.hip`` full
fills, ``nw_strip.hip`` score-only fills); there is no CPU fallback: if the library is missing or
no GPU is visible, GPU entry points raise.

Mirrors the reference's registry (src/nw_algorithm.cpp:48-69): an ``NwAlgorithm`` is an
{align, trace, hash} triple; the plain family pairs with Trace1/Hash1, the sparse (mlsp)
family with Trace2/Hash2.
"""
from __future__ import annotations

import ctypes
import dataclasses
import os
from typing import Callable, Dict, Optional, Sequence, Tuple

import numpy as np

__all__ = [
    "NwStat", "NwError", "lib", "Engine", "AlignResult", "SparseResult", "PairDev",
    "NwAlgorithm", "get_nw_algorithm_map", "hash_full", "trace_full", "trace_sparse", "hash_sparse",
    "sparse_align_cost", "sparse_tile_by",
]

_PKG = os.path.dirname(os.path.abspath(__file__))
_SO = os.environ.get("GSA_LIB") or os.path.join(_PKG, "libgsa.so")  # GSA_LIB: diagnostic builds only
_LIB = None


class NwStat:
    """NwStat (src/run_types.hpp:12-24)."""
    success = 0
    helpMenuRequested = 1
    errorCudaGeneral = 2
    errorMemoryAllocation = 3
    errorMemoryTransfer = 4
    errorKernelFailure = 5
    errorIoStream = 6
    errorInvalidFormat = 7
    errorInvalidValue = 8
    errorInvalidResult = 9
    names = {0: "success", 1: "helpMenuRequested", 2: "errorCudaGeneral", 3: "errorMemoryAllocation",
             4: "errorMemoryTransfer", 5: "errorKernelFailure", 6: "errorIoStream", 7: "errorInvalidFormat",
             8: "errorInvalidValue", 9: "errorInvalidResult"}


class NwError(RuntimeError):
    def __init__(self, stat: int, where: str, hip_error: int = 0):
        self.stat = stat
        self.hip_error = hip_error
        super().__init__(f"{where}: {NwStat.names.get(stat, stat)} (hipError {hip_error})")


class _Laps(ctypes.Structure):
    _fields_ = [("alloc", ctypes.c_float), ("cpy_dev", ctypes.c_float), ("init_hdr", ctypes.c_float),
                ("calc", ctypes.c_float), ("cpy_host", ctypes.c_float), ("calc_kernel_ms", ctypes.c_float)]

    def as_dict(self):
        return {"align.alloc": self.alloc, "align.cpy_dev": self.cpy_dev, "align.init_hdr": self.init_hdr,
                "align.calc": self.calc, "align.cpy_host": self.cpy_host, "calc_kernel_ms": self.calc_kernel_ms}


class SparseGeom(ctypes.Structure):
    _fields_ = [("tileBx", ctypes.c_int32), ("tileBy", ctypes.c_int32), ("tileHdrMatRows", ctypes.c_int32),
                ("tileHdrMatCols", ctypes.c_int32), ("tileHrowLen", ctypes.c_int32), ("tileHcolLen", ctypes.c_int32),
                ("hrowElems", ctypes.c_int64), ("hcolElems", ctypes.c_int64)]


class PairDev(ctypes.Structure):
    """gsa_pair_dev (include/gsa.h): device pointers of one pair of a batched fill."""
    _fields_ = [("seqY", ctypes.c_void_p), ("adjrows", ctypes.c_int32), ("seqX", ctypes.c_void_p),
                ("adjcols", ctypes.c_int32), ("score", ctypes.c_void_p), ("tileHrowMat", ctypes.c_void_p),
                ("tileHcolMat", ctypes.c_void_p)]


class CheckResult(ctypes.Structure):
    """gsa_check_result (include/gsa.h): outcome of a device-side verification."""
    _fields_ = [("checked", ctypes.c_int64), ("mismatches", ctypes.c_int64), ("first", ctypes.c_int64)]

    def as_dict(self):
        return {"checked": int(self.checked), "mismatches": int(self.mismatches), "first": int(self.first)}


class MemStats(ctypes.Structure):
    """gsa_mem_stats: the reference's NwAlgResult peak-alloc columns (nwalign_shared.cpp:5-25)."""
    _fields_ = [("glmem_peak_allocs", ctypes.c_int64), ("shmem_peak_allocs", ctypes.c_int64),
                ("locmem_peak_allocs", ctypes.c_int64), ("regmem_peak_allocs", ctypes.c_int64)]

    def as_dict(self):
        return {k: int(getattr(self, k)) for k, _ in self._fields_}


class FullTiming(ctypes.Structure):
    """gsa_full_timing (include/gsa.h): pass times and pass 2's effective shader clock."""
    _fields_ = [("pass1_ms", ctypes.c_float), ("pass2_ms", ctypes.c_float),
                ("clock_ghz_median", ctypes.c_float), ("clock_ghz_mean", ctypes.c_float),
                ("workgroups", ctypes.c_int64), ("fused", ctypes.c_int32), ("groups", ctypes.c_int32)]


class ScoreResult(ctypes.Structure):
    """gsa_score_result (include/gsa.h)."""
    _fields_ = [("score", ctypes.c_int32), ("i_end", ctypes.c_int64), ("j_end", ctypes.c_int64),
                ("calc_kernel_ms", ctypes.c_float)]


_LAPFN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_char_p)  # gsa_lap_fn
_i32p = ctypes.POINTER(ctypes.c_int32)
_vp = ctypes.c_void_p
_i32 = ctypes.c_int32
_i64 = ctypes.c_int64

# symbol -> (restype, argtypes); every function declared in include/gsa.h
SIGNATURES = {
    "gsa_ctx_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(_vp)]),
    "gsa_ctx_destroy": (None, [_vp]),
    "gsa_last_hip_error": (ctypes.c_int, [_vp]),
    "gsa_device_cu_count": (ctypes.c_int, [_vp]),
    "gsa_version": (ctypes.c_char_p, []),
    "gsa_debug_stamps": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64)]),
    "gsa_set_lap_callback": (ctypes.c_int, [_vp, _vp, _vp]),
    "gsa_set_knob": (ctypes.c_int, [_vp, ctypes.c_char_p, ctypes.c_char_p]),
    "gsa_set_full_timing": (ctypes.c_int, [_vp, _i32]),
    "gsa_last_full_timing": (ctypes.c_int, [_vp, ctypes.POINTER(FullTiming)]),
    "gsa_sparse_tile_by": (_i32, []),
    "gsa_sparse_geometry": (ctypes.c_int, [_i32, _i32, _i32, ctypes.POINTER(SparseGeom)]),
    "gsa_fill_full_dev": (ctypes.c_int, [_vp, _vp, _i32, _vp, _i32, _vp, _i32, _i32, _vp, _vp]),
    "gsa_fill_sparse_dev": (ctypes.c_int, [_vp, _vp, _i32, _vp, _i32, _vp, _i32, _i32, _i32, _vp, _vp, _vp]),
    "gsa_sync": (ctypes.c_int, [_vp, _vp]),
    "gsa_set_watchdog": (ctypes.c_int, [_vp, _i64]),
    "gsa_mem_stats_get": (ctypes.c_int, [_vp, ctypes.POINTER(MemStats)]),
    "gsa_mem_stats_reset": (ctypes.c_int, [_vp]),
    "gsa_fill_full_batch_dev": (ctypes.c_int, [_vp, _i32, ctypes.POINTER(PairDev), _vp, _i32, _i32, _vp]),
    "gsa_full_pitch": (_i32, [_i32]),
    "gsa_full_base_offset": (_i32, []),
    "gsa_fill_full_pitched_dev": (ctypes.c_int, [_vp, _vp, _i32, _vp, _i32, _vp, _i32, _i32, _vp, _i32, _vp]),
    "gsa_fill_full_batch_pitched_dev": (ctypes.c_int, [_vp, _i32, ctypes.POINTER(PairDev), _i32p, _vp, _i32, _i32,
                                                       _vp]),
    "gsa_fill_sparse_batch_dev": (ctypes.c_int, [_vp, _i32, ctypes.POINTER(PairDev), _vp, _i32, _i32, _i32, _vp]),
    "gsa_align_full": (ctypes.c_int, [_vp, _i32p, _i32, _i32p, _i32, _i32p, _i32, _i32, _i32p, _i32p,
                                      ctypes.POINTER(_Laps)]),
    "gsa_align_sparse": (ctypes.c_int, [_vp, _i32p, _i32, _i32p, _i32, _i32p, _i32, _i32, _i32, _i32p, _i32p,
                                        ctypes.POINTER(SparseGeom), _i32p, ctypes.POINTER(_Laps)]),
    "gsa_align_sparse_pt": (ctypes.c_int, [_vp, _i32p, _i32, _i32p, _i32, _i32p, _i32, _i32, _i32, _i32p, _i32p,
                                           ctypes.POINTER(SparseGeom), _i32p, ctypes.POINTER(_Laps)]),
    "gsa_hash_full": (ctypes.c_uint32, [_i32p, _i32, _i32]),
    "gsa_trace_full": (ctypes.c_int, [_i32p, _i32p, _i32, _i32p, _i32, ctypes.c_char_p, _i64,
                                      ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_uint32)]),
    "gsa_trace_sparse": (ctypes.c_int, [_i32p, _i32p, ctypes.POINTER(SparseGeom), _i32p, _i32, _i32p, _i32, _i32p,
                                        _i32, _i32, ctypes.c_char_p, _i64, ctypes.POINTER(ctypes.c_int64),
                                        ctypes.POINTER(ctypes.c_uint32), _i32p]),
    "gsa_hash_sparse": (ctypes.c_uint32, [_i32p, _i32p, ctypes.POINTER(SparseGeom), _i32p, _i32, _i32p, _i32, _i32p,
                                          _i32, _i32]),
    "gsa_sparse_align_cost": (_i32, [_i32p, _i32p, ctypes.POINTER(SparseGeom), _i32p, _i32, _i32p, _i32, _i32p,
                                     _i32, _i32]),
    "gsa_check_sparse_dev": (ctypes.c_int, [_vp, _vp, _i32, _vp, _i32, _vp, _i32, _i32, ctypes.POINTER(SparseGeom),
                                            _vp, _vp, ctypes.POINTER(CheckResult), _vp]),
    "gsa_check_full_dev": (ctypes.c_int, [_vp, _vp, _i32, _vp, _i32, _vp, _i32, _i32, _vp,
                                          ctypes.POINTER(CheckResult), _vp]),
    "gsa_check_full_pitched_dev": (ctypes.c_int, [_vp, _vp, _i32, _vp, _i32, _vp, _i32, _i32, _vp, _i32,
                                                  ctypes.POINTER(CheckResult), _vp]),
    "gsa_hash_full_dev": (ctypes.c_int, [_vp, _vp, _i32, _i32, _i32, ctypes.POINTER(ctypes.c_uint32), _vp]),
    "gsa_trace_full_dev": (ctypes.c_int, [_vp, _vp, _i32, _vp, _i32, _vp, _i32, ctypes.c_char_p, _i64,
                                          ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_uint32), _i32p,
                                          _vp]),
    "gsa_score_dev": (ctypes.c_int, [_vp, _vp, _i32, _vp, _i32, _vp, _i32, _i32, _i32, _i32,
                                     ctypes.POINTER(ScoreResult), _vp]),
    "gsa_score": (ctypes.c_int, [_vp, _i32p, _i32, _i32p, _i32, _i32p, _i32, _i32, _i32, _i32,
                                 ctypes.POINTER(ScoreResult), ctypes.POINTER(_Laps)]),
    "gsa_trace_sparse_dev": (ctypes.c_int, [_vp, _vp, _i32, _vp, _i32, _vp, _i32, _i32, ctypes.POINTER(SparseGeom),
                                            _vp, _vp, ctypes.c_char_p, _i64, ctypes.POINTER(ctypes.c_int64),
                                            ctypes.POINTER(ctypes.c_uint32), _i32p, _vp]),
}


def lib():
    """Load libgsa.so.  Raises if it has not been built: there is no fallback path."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(_SO):
            raise ImportError(f"{_SO} missing: run __graft_entry__.build() (hipcc --offload-arch=gfx950)")
        L = ctypes.CDLL(_SO)
        for name, (res, args) in SIGNATURES.items():
            if os.environ.get("GSA_LIB") and not hasattr(L, name):
                continue  # diagnostic builds of older revisions may lack newer entry points
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _LIB = L
    return _LIB


def _p(a: np.ndarray):
    assert a.dtype == np.int32 and a.flags["C_CONTIGUOUS"], (a.dtype, a.flags)
    return a.ctypes.data_as(_i32p)


def _c32(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.int32)


def sparse_tile_by() -> int:
    return int(lib().gsa_sparse_tile_by())


def full_pitch(adjcols: int) -> int:
    """Row pitch (ints) of the fastest device layout of a full matrix (gsa_full_pitch: = 1 mod 32)."""
    return int(lib().gsa_full_pitch(adjcols))


def full_base_offset() -> int:
    """Ints from a 128-byte boundary to cell (0, 0) of that layout (cell (1, 0) on the boundary)."""
    return int(lib().gsa_full_base_offset())


def sparse_geometry(adjrows: int, adjcols: int, tileBx: int) -> SparseGeom:
    g = SparseGeom()
    st = lib().gsa_sparse_geometry(adjrows, adjcols, tileBx, ctypes.byref(g))
    if st != NwStat.success:
        raise NwError(st, "gsa_sparse_geometry")
    return g


@dataclasses.dataclass
class AlignResult:
    score: np.ndarray  # (adjrows, adjcols) int32
    align_cost: int
    laps: dict


@dataclasses.dataclass
class SparseResult:
    hrow: np.ndarray
    hcol: np.ndarray
    geom: SparseGeom
    align_cost: int
    laps: dict

    @property
    def trows(self):
        return self.geom.tileHdrMatRows

    @property
    def tcols(self):
        return self.geom.tileHdrMatCols


class Engine:
    """One device context (initNwInput equivalent, src/benchmark.cpp:175-223)."""

    def __init__(self, device: int = 0):
        self.device = device
        h = _vp()
        st = lib().gsa_ctx_create(device, ctypes.byref(h))
        if st != NwStat.success:
            raise NwError(st, f"gsa_ctx_create(device={device})")
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            lib().gsa_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    @property
    def cu_count(self) -> int:
        return int(lib().gsa_device_cu_count(self._h))

    def _check(self, st, where):
        if st != NwStat.success:
            raise NwError(st, where, int(lib().gsa_last_hip_error(self._h)))

    # -- NwAlignFn equivalents (host buffers) -------------------------------------------
    def align_full(self, seqY, seqX, subst, gapo: int) -> AlignResult:
        """Full int32 score matrix (the gpu3..gpu6 family's nw.score)."""
        seqY, seqX, subst = _c32(seqY), _c32(seqX), _c32(subst)
        substsz = int(round(np.sqrt(subst.size)))
        score = np.empty((len(seqY), len(seqX)), dtype=np.int32)
        cost = ctypes.c_int32(0)
        laps = _Laps()
        st = lib().gsa_align_full(self._h, _p(seqY), len(seqY), _p(seqX), len(seqX), _p(subst), substsz, gapo,
                                  _p(score), ctypes.byref(cost), ctypes.byref(laps))
        self._check(st, "gsa_align_full")
        return AlignResult(score, int(cost.value), laps.as_dict())

    def align_sparse(self, seqY, seqX, subst, gapo: int, tileBx: int = 256, overlap: bool = False) -> SparseResult:
        """Tile-header (mlsp) representation (the gpu7..gpu9 family's tileHrowMat/tileHcolMat).
        overlap=True: mlsppt, the copy-back runs tile row by tile row during the fill."""
        seqY, seqX, subst = _c32(seqY), _c32(seqX), _c32(subst)
        substsz = int(round(np.sqrt(subst.size)))
        geom = sparse_geometry(len(seqY), len(seqX), tileBx)
        hrow = np.empty(geom.hrowElems, dtype=np.int32)
        hcol = np.empty(geom.hcolElems, dtype=np.int32)
        cost = ctypes.c_int32(0)
        laps = _Laps()
        fn = lib().gsa_align_sparse_pt if overlap else lib().gsa_align_sparse
        st = fn(self._h, _p(seqY), len(seqY), _p(seqX), len(seqX), _p(subst), substsz, gapo, tileBx, _p(hrow),
                _p(hcol), ctypes.byref(geom), ctypes.byref(cost), ctypes.byref(laps))
        self._check(st, "gsa_align_sparse_pt" if overlap else "gsa_align_sparse")
        return SparseResult(hrow, hcol, geom, int(cost.value), laps.as_dict())

    # -- hot path on device-resident buffers (torch tensors or raw pointers) -------------
    def fill_full_dev(self, seqY_ptr: int, adjrows: int, seqX_ptr: int, adjcols: int, subst_ptr: int, substsz: int,
                      gapo: int, score_ptr: int, stream: Optional[int] = None, ld: Optional[int] = None):
        """Full matrix into device memory; ld = row pitch in ints (None: unpadded, adjcols)."""
        if ld is None:
            st = lib().gsa_fill_full_dev(self._h, seqY_ptr, adjrows, seqX_ptr, adjcols, subst_ptr, substsz, gapo,
                                         score_ptr, stream)
            self._check(st, "gsa_fill_full_dev")
        else:
            st = lib().gsa_fill_full_pitched_dev(self._h, seqY_ptr, adjrows, seqX_ptr, adjcols, subst_ptr, substsz,
                                                 gapo, score_ptr, int(ld), stream)
            self._check(st, "gsa_fill_full_pitched_dev")

    def fill_sparse_dev(self, seqY_ptr: int, adjrows: int, seqX_ptr: int, adjcols: int, subst_ptr: int,
                        substsz: int, gapo: int, tileBx: int, hrow_ptr: int, hcol_ptr: int,
                        stream: Optional[int] = None):
        st = lib().gsa_fill_sparse_dev(self._h, seqY_ptr, adjrows, seqX_ptr, adjcols, subst_ptr, substsz, gapo,
                                       tileBx, hrow_ptr, hcol_ptr, stream)
        self._check(st, "gsa_fill_sparse_dev")

    def fill_batch_dev(self, pairs, subst_ptr: int, substsz: int, gapo: int, mode: str = "sparse",
                       tileBx: int = 256, stream: Optional[int] = None, lds: Optional[Sequence[int]] = None):
        """One persistent launch over many pairs.  `pairs`: sequence of (seqY_ptr, adjrows,
        seqX_ptr, adjcols, out) with out = score_ptr (full) or (hrow_ptr, hcol_ptr) (sparse);
        lds: full matrices' row pitches (None: unpadded)."""
        arr = (PairDev * len(pairs))()
        for k, (yp, ar, xp, ac, out) in enumerate(pairs):
            arr[k].seqY, arr[k].adjrows, arr[k].seqX, arr[k].adjcols = yp, ar, xp, ac
            if mode == "sparse":
                arr[k].tileHrowMat, arr[k].tileHcolMat = out
            else:
                arr[k].score = out
        if mode == "sparse":
            st = lib().gsa_fill_sparse_batch_dev(self._h, len(pairs), arr, subst_ptr, substsz, gapo, tileBx, stream)
        elif lds is None:
            st = lib().gsa_fill_full_batch_dev(self._h, len(pairs), arr, subst_ptr, substsz, gapo, stream)
        else:
            la = _c32(list(lds))
            st = lib().gsa_fill_full_batch_pitched_dev(self._h, len(pairs), arr, _p(la), subst_ptr, substsz, gapo,
                                                       stream)
        self._check(st, "gsa_fill_%s_batch_dev" % mode)

    def sync(self, stream: Optional[int] = None):
        """Wait for `stream`; raises NwError if a hand-off of ANY fill enqueued since the last
        sync gave up (the error word is sticky until this call clears it)."""
        self._check(lib().gsa_sync(self._h, stream), "gsa_sync")

    def debug_stamps(self):
        """The stamps of the last launch made under GSA_STAMPS=1 (gsa_debug_stamps), uint64: a fused
        full fill's [realtime start, end, shader clock start, end] per pass-1 strip, then [claimed,
        ready, done] per expansion task; a K-rows fill's strip ledger [realtime start, end, clock
        start, end, cycles waiting, waits, 4 block spans (diagnostic builds)] per strip; empty if
        none were recorded."""
        import numpy as np
        n = ctypes.c_int64(0)
        self._check(lib().gsa_debug_stamps(self._h, None, 0, ctypes.byref(n)), "gsa_debug_stamps")
        out = np.zeros(n.value, dtype=np.uint64)
        if n.value:
            self._check(lib().gsa_debug_stamps(self._h, out.ctypes.data, n.value, ctypes.byref(n)), "gsa_debug_stamps")
        return out

    def set_full_timing(self, on: bool = True):
        """Events around the passes of every two-pass full fill and pass 2's clock stamps
        (gsa_set_full_timing; a measurement aid)."""
        self._check(lib().gsa_set_full_timing(self._h, 1 if on else 0), "gsa_set_full_timing")

    def last_full_timing(self) -> dict:
        """The last timed full fill (gsa_last_full_timing): pass1_ms, pass2_ms (HIP events; a fused
        fill: pass1_ms None, the launch in pass2_ms), pass 2's effective clock in GHz (median over
        workgroups and cycle-weighted mean of s_memtime / s_memrealtime), waits for that fill."""
        t = FullTiming()
        self._check(lib().gsa_last_full_timing(self._h, ctypes.byref(t)), "gsa_last_full_timing")
        f = lambda v: None if v < 0 else round(float(v), 4)
        return {"pass1_ms": f(t.pass1_ms), "pass2_ms": f(t.pass2_ms), "clock_ghz_median": f(t.clock_ghz_median),
                "clock_ghz_mean": f(t.clock_ghz_mean), "clock_workgroups": int(t.workgroups), "fused": bool(t.fused),
                "pipelined_groups": int(t.groups)}

    def set_knob(self, name: str, value: Optional[str]):
        """Set a measurement / test switch (GSA_FULL_KERNEL, GSA_KROW_NS, ...) for this context
        (gsa_set_knob); None unsets it.  A context takes the knobs from the environment once, when
        it is created."""
        self._check(lib().gsa_set_knob(self._h, name.encode(), None if value is None else str(value).encode()),
                    "gsa_set_knob")

    def set_lap_callback(self, fn: Optional[Callable[[str], None]]):
        """fn(lap_name) at every phase boundary of the host-buffer entry points (align_full,
        align_sparse, score): gsa_set_lap_callback, the hook an adapter uses to drive the
        reference's Stopwatch::lap (src/stopwatch.hpp:19).  None removes it."""
        if fn is None:
            self._lapcb = None
            self._check(lib().gsa_set_lap_callback(self._h, None, None), "gsa_set_lap_callback")
            return
        cb = _LAPFN(lambda _user, name: fn(name.decode()))
        self._check(lib().gsa_set_lap_callback(self._h, ctypes.cast(cb, _vp), None), "gsa_set_lap_callback")
        self._lapcb = cb  # keep the thunk alive while the library holds it

    def set_watchdog(self, microseconds: int):
        """No-progress limit of every wait inside later fills (default 1 s)."""
        self._check(lib().gsa_set_watchdog(self._h, int(microseconds)), "gsa_set_watchdog")

    def mem_stats(self) -> dict:
        m = MemStats()
        self._check(lib().gsa_mem_stats_get(self._h, ctypes.byref(m)), "gsa_mem_stats_get")
        return m.as_dict()

    def reset_mem_stats(self):
        self._check(lib().gsa_mem_stats_reset(self._h), "gsa_mem_stats_reset")

    # -- score-only NW / SW, linear or affine gaps (BASELINE configs[4]) -----------------
    def score(self, seqY, seqX, subst, gapo: int, gape: Optional[int] = None, local: bool = False) -> dict:
        """Score-only alignment (host buffers): {"score", "i_end", "j_end", "laps"}; gape
        defaults to gapo (linear gaps; global + linear = the reference's NW-LG align_cost)."""
        seqY, seqX, subst = _c32(seqY), _c32(seqX), _c32(subst)
        substsz = int(round(np.sqrt(subst.size)))
        r = ScoreResult()
        laps = _Laps()
        st = lib().gsa_score(self._h, _p(seqY), len(seqY), _p(seqX), len(seqX), _p(subst), substsz, gapo,
                             gapo if gape is None else gape, int(local), ctypes.byref(r), ctypes.byref(laps))
        self._check(st, "gsa_score")
        return {"score": int(r.score), "i_end": int(r.i_end), "j_end": int(r.j_end), "laps": laps.as_dict()}

    def score_dev(self, seqY_ptr: int, adjrows: int, seqX_ptr: int, adjcols: int, subst_ptr: int, substsz: int,
                  gapo: int, gape: int, local: bool = False, stream: Optional[int] = None) -> dict:
        r = ScoreResult()
        st = lib().gsa_score_dev(self._h, seqY_ptr, adjrows, seqX_ptr, adjcols, subst_ptr, substsz, gapo, gape,
                                 int(local), ctypes.byref(r), stream)
        self._check(st, "gsa_score_dev")
        return {"score": int(r.score), "i_end": int(r.i_end), "j_end": int(r.j_end),
                "kernel_ms": float(r.calc_kernel_ms)}

    # -- device-side verification ---------------------------------------

    def check_sparse_dev(self, seqY_ptr: int, adjrows: int, seqX_ptr: int, adjcols: int, subst_ptr: int,
                         substsz: int, gapo: int, geom: SparseGeom, hrow_ptr: int, hcol_ptr: int,
                         stream: Optional[int] = None) -> dict:
        """Every header value of a sparse fill against the recurrence (tile consistency);
        synchronous.  Returns {"checked", "mismatches", "first"}."""
        r = CheckResult()
        st = lib().gsa_check_sparse_dev(self._h, seqY_ptr, adjrows, seqX_ptr, adjcols, subst_ptr, substsz, gapo,
                                        ctypes.byref(geom), hrow_ptr, hcol_ptr, ctypes.byref(r), stream)
        self._check(st, "gsa_check_sparse_dev")
        return r.as_dict()

    def trace_sparse_dev(self, seqY_ptr: int, adjrows: int, seqX_ptr: int, adjcols: int, subst_ptr: int,
                         substsz: int, gapo: int, geom: SparseGeom, hrow_ptr: int, hcol_ptr: int,
                         stream: Optional[int] = None) -> Tuple[int, str, int]:
        """NwTrace2_Sparse on the device (headers stay in HBM): (trace_hash, edit string,
        align_cost), identical to trace_sparse()."""
        cap = 8 * (adjrows + adjcols) + 64  # run-length string: <= 2 chars per move, digits reversed
        buf = ctypes.create_string_buffer(cap)
        n = ctypes.c_int64(0)
        h = ctypes.c_uint32(0)
        cost = ctypes.c_int32(0)
        st = lib().gsa_trace_sparse_dev(self._h, seqY_ptr, adjrows, seqX_ptr, adjcols, subst_ptr, substsz, gapo,
                                        ctypes.byref(geom), hrow_ptr, hcol_ptr, buf, cap, ctypes.byref(n),
                                        ctypes.byref(h), ctypes.byref(cost), stream)
        self._check(st, "gsa_trace_sparse_dev")
        return int(h.value), buf.raw[:n.value].decode(), int(cost.value)

    def check_full_dev(self, seqY_ptr: int, adjrows: int, seqX_ptr: int, adjcols: int, subst_ptr: int,
                       substsz: int, gapo: int, score_ptr: int, stream: Optional[int] = None,
                       ld: Optional[int] = None) -> dict:
        """Every cell of a full matrix against its stored neighbours; synchronous.  ld: row pitch
        (None: unpadded)."""
        r = CheckResult()
        if ld is None:
            st = lib().gsa_check_full_dev(self._h, seqY_ptr, adjrows, seqX_ptr, adjcols, subst_ptr, substsz, gapo,
                                          score_ptr, ctypes.byref(r), stream)
        else:
            st = lib().gsa_check_full_pitched_dev(self._h, seqY_ptr, adjrows, seqX_ptr, adjcols, subst_ptr, substsz,
                                                  gapo, score_ptr, int(ld), ctypes.byref(r), stream)
        self._check(st, "gsa_check_full_dev" if ld is None else "gsa_check_full_pitched_dev")
        return r.as_dict()

    def hash_full_dev(self, score_ptr: int, adjrows: int, adjcols: int, ld: Optional[int] = None,
                      stream: Optional[int] = None) -> int:
        """NwHash1_Plain of a device-resident full matrix (gsa_hash_full_dev); equals hash_full()
        of its host copy."""
        h = ctypes.c_uint32(0)
        st = lib().gsa_hash_full_dev(self._h, score_ptr, adjrows, adjcols, adjcols if ld is None else int(ld),
                                     ctypes.byref(h), stream)
        self._check(st, "gsa_hash_full_dev")
        return int(h.value)

    def trace_full_dev(self, seqY_ptr: int, adjrows: int, seqX_ptr: int, adjcols: int, score_ptr: int,
                       ld: Optional[int] = None, stream: Optional[int] = None) -> Tuple[int, str, int]:
        """NwTrace1_Plain of a device-resident full matrix (gsa_trace_full_dev): (trace_hash, edit
        string, align_cost), equal to trace_full() of its host copy."""
        cap = 8 * (adjrows + adjcols) + 64
        buf = ctypes.create_string_buffer(cap)
        n = ctypes.c_int64(0)
        h = ctypes.c_uint32(0)
        cost = ctypes.c_int32(0)
        st = lib().gsa_trace_full_dev(self._h, seqY_ptr, adjrows, seqX_ptr, adjcols, score_ptr,
                                      adjcols if ld is None else int(ld), buf, cap, ctypes.byref(n), ctypes.byref(h),
                                      ctypes.byref(cost), stream)
        self._check(st, "gsa_trace_full_dev")
        return int(h.value), buf.raw[:n.value].decode(), int(cost.value)


# ---- host consumers (the reference's L4) ----------------------------------------------

def hash_full(score: np.ndarray) -> int:
    """NwHash1_Plain (src/nwtrace1_plain.cpp:133-154)."""
    score = _c32(score)
    return int(lib().gsa_hash_full(_p(score), score.shape[0], score.shape[1]))


def trace_full(score: np.ndarray, seqY, seqX) -> Tuple[int, str]:
    """NwTrace1_Plain (src/nwtrace1_plain.cpp:6-131) -> (trace_hash, edit_trace)."""
    score, seqY, seqX = _c32(score), _c32(seqY), _c32(seqX)
    cap = 8 * (len(seqY) + len(seqX)) + 64
    buf = ctypes.create_string_buffer(cap)
    n = ctypes.c_int64(0)
    h = ctypes.c_uint32(0)
    st = lib().gsa_trace_full(_p(score), _p(seqY), len(seqY), _p(seqX), len(seqX), buf, cap, ctypes.byref(n),
                              ctypes.byref(h))
    if st != NwStat.success:
        raise NwError(st, "gsa_trace_full")
    return int(h.value), buf.raw[:n.value].decode()


def trace_sparse(res: SparseResult, seqY, seqX, subst, gapo: int) -> Tuple[int, str, int]:
    """NwTrace2_Sparse (src/nwtrace2_sparse.cpp:102-257) -> (trace_hash, edit_trace, align_cost)."""
    seqY, seqX, subst = _c32(seqY), _c32(seqX), _c32(subst)
    substsz = int(round(np.sqrt(subst.size)))
    cap = 8 * (len(seqY) + len(seqX)) + 64
    buf = ctypes.create_string_buffer(cap)
    n = ctypes.c_int64(0)
    h = ctypes.c_uint32(0)
    cost = ctypes.c_int32(0)
    st = lib().gsa_trace_sparse(_p(_c32(res.hrow)), _p(_c32(res.hcol)), ctypes.byref(res.geom), _p(seqY), len(seqY),
                                _p(seqX), len(seqX), _p(subst), substsz, gapo, buf, cap, ctypes.byref(n),
                                ctypes.byref(h), ctypes.byref(cost))
    if st != NwStat.success:
        raise NwError(st, "gsa_trace_sparse")
    return int(h.value), buf.raw[:n.value].decode(), int(cost.value)


def hash_sparse(res: SparseResult, seqY, seqX, subst, gapo: int) -> int:
    """NwHash2_Sparse (src/nwtrace2_sparse.cpp:263-340)."""
    seqY, seqX, subst = _c32(seqY), _c32(seqX), _c32(subst)
    substsz = int(round(np.sqrt(subst.size)))
    return int(lib().gsa_hash_sparse(_p(_c32(res.hrow)), _p(_c32(res.hcol)), ctypes.byref(res.geom), _p(seqY),
                                     len(seqY), _p(seqX), len(seqX), _p(subst), substsz, gapo))


def sparse_align_cost(res: SparseResult, seqY, seqX, subst, gapo: int) -> int:
    seqY, seqX, subst = _c32(seqY), _c32(seqX), _c32(subst)
    substsz = int(round(np.sqrt(subst.size)))
    return int(lib().gsa_sparse_align_cost(_p(_c32(res.hrow)), _p(_c32(res.hcol)), ctypes.byref(res.geom),
                                           _p(seqY), len(seqY), _p(seqX), len(seqX), _p(subst), substsz, gapo))


# ---- the registry (src/nw_algorithm.hpp:8-42) --------------------------------------------

@dataclasses.dataclass
class NwResult:
    """The fields of NwAlgResult the driver verifies (src/benchmark.cpp:120-147)."""
    align_cost: int = 0
    score_hash: int = 0
    trace_hash: int = 0
    edit_trace: str = ""
    laps: dict = dataclasses.field(default_factory=dict)
    payload: object = None


@dataclasses.dataclass
class NwAlgorithm:
    name: str
    align: Callable
    trace: Callable
    hash: Callable
    params: Dict[str, list] = dataclasses.field(default_factory=dict)


def _align_plain(engine: Engine, seqY, seqX, subst, gapo, **_):
    r = engine.align_full(seqY, seqX, subst, gapo)
    return NwResult(align_cost=r.align_cost, laps=r.laps, payload=r)


def _align_mlsp(engine: Engine, seqY, seqX, subst, gapo, tileBx=256, **_):
    r = engine.align_sparse(seqY, seqX, subst, gapo, tileBx=tileBx)
    return NwResult(align_cost=r.align_cost, laps=r.laps, payload=r)


def _align_mlsppt(engine: Engine, seqY, seqX, subst, gapo, tileBx=256, **_):
    r = engine.align_sparse(seqY, seqX, subst, gapo, tileBx=tileBx, overlap=True)
    return NwResult(align_cost=r.align_cost, laps=r.laps, payload=r)


def _trace1(res: NwResult, seqY, seqX, subst, gapo):
    res.trace_hash, res.edit_trace = trace_full(res.payload.score, seqY, seqX)


def _hash1(res: NwResult, seqY, seqX, subst, gapo):
    res.score_hash = hash_full(res.payload.score)


def _trace2(res: NwResult, seqY, seqX, subst, gapo):
    res.trace_hash, res.edit_trace, _ = trace_sparse(res.payload, seqY, seqX, subst, gapo)


def _hash2(res: NwResult, seqY, seqX, subst, gapo):
    res.score_hash = hash_sparse(res.payload, seqY, seqX, subst, gapo)


def get_nw_algorithm_map() -> Dict[str, NwAlgorithm]:
    """getNwAlgorithmMap (src/nw_algorithm.cpp:48-69) for this engine.

    The reference's GPU family names resolve to the MI355X wavefront kernels: the
    full-matrix names (gpu3..gpu6) to the plain fill with Trace1/Hash1, the mlsp names
    (gpu7..gpu9) to the tile-header fill with Trace2/Hash2."""
    plain = ["NwAlign_Amd_Strip_Full", "NwAlign_Gpu3_Ml_DiagDiag", "NwAlign_Gpu4_Ml_DiagDiag2Pass",
             "NwAlign_Gpu5_Coop_DiagDiag", "NwAlign_Gpu6_Coop_DiagDiag2Pass"]
    mlsp = ["NwAlign_Amd_Strip_Mlsp", "NwAlign_Gpu7_Mlsp_DiagDiag", "NwAlign_Gpu8_Mlsp_DiagDiag",
            "NwAlign_Gpu9_Mlsp_DiagDiagDiag"]
    m = {n: NwAlgorithm(n, _align_plain, _trace1, _hash1) for n in plain}
    m.update({n: NwAlgorithm(n, _align_mlsp, _trace2, _hash2, {"tileBx": [256]}) for n in mlsp})
    # mlsppt (the reference's README.md:39 names it, never implemented): copy-back overlapped
    m["NwAlign_Amd_Strip_Mlsppt"] = NwAlgorithm("NwAlign_Amd_Strip_Mlsppt", _align_mlsppt, _trace2, _hash2,
                                                {"tileBx": [256]})
    return m
