"""Host-buffer entry points on the device: the lap callback (gsa_set_lap_callback, the hook the
NwAlignFn adapter uses to drive the reference's Stopwatch::lap, src/stopwatch.hpp:19), and the
boundary's fallbacks and rejections around the score and trace entry points."""
import numpy as np
import pytest

import gpuseqalign_amd as gsa
from tests._data import random_pair, related_pair

pytestmark = pytest.mark.gpu


def _dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.int32)).to("cuda:0")


# the reference's lap order (nwalign_gpu3_ml_diagdiag.cu:329-593, nwalign_gpu9_mlsp_diagdiagdiag.cu:435-719)
FULL = ["align.alloc", "align.cpy_dev", "align.init_hdr", "align.calc", "align.cpy_host"]
SPARSE = FULL + ["align.calc"]


@pytest.mark.parametrize("what", ["full", "mlsp", "mlsppt", "score"])
def test_lap_callback_order_and_totals(golden, what):
    import time
    Y, X = random_pair(2100, 2600, 11)
    sub = golden.blosum62
    names, stamps = [], []
    with gsa.Engine(0) as eng:
        eng.set_lap_callback(lambda n: (names.append(n), stamps.append(time.perf_counter())))
        t0 = time.perf_counter()
        if what == "full":
            r = eng.align_full(Y, X, sub, -11)
            laps = r.laps
        elif what == "score":
            r = eng.score(Y, X, sub, -11, -1, False)
            laps = r["laps"]
        else:
            r = eng.align_sparse(Y, X, sub, -11, tileBx=256, overlap=(what == "mlsppt"))
            laps = r.laps
        t1 = time.perf_counter()
        want = {"full": FULL, "score": ["align.alloc", "align.cpy_dev", "align.calc"]}.get(what, SPARSE)
        assert names == want
        # the callback's intervals cover the call, and its align.calc is at least the fill's lap
        assert t0 <= stamps[0] and stamps[-1] <= t1
        calc = sum(b - a for a, b, n in zip([t0] + stamps[:-1], stamps, names) if n == "align.calc") * 1e3
        assert calc >= 0.9 * laps["align.calc"] - 0.05
        eng.set_lap_callback(None)
        eng.align_full(Y[:50], X[:60], sub, -11)
        assert len(names) == len(want)  # removed: no further calls


def test_trace_band_budget_fallback(engine, golden, monkeypatch, knobs):
    """The band precompute is a speed-up only: with no memory budget for it (as when its buffers
    cannot be allocated) the device walk runs alone and still equals the host Trace2."""
    import torch
    Y, X = related_pair(5000, 5300)
    sub = golden.blosum62
    geom = gsa.sparse_geometry(len(Y), len(X), 256)
    y, x, s = _dev(Y), _dev(X), _dev(sub)
    hr = torch.empty(geom.hrowElems, dtype=torch.int32, device="cuda:0")
    hc = torch.empty(geom.hcolElems, dtype=torch.int32, device="cuda:0")
    args = (y.data_ptr(), len(Y), x.data_ptr(), len(X), s.data_ptr(), 25, -11)
    engine.fill_sparse_dev(*args, 256, hr.data_ptr(), hc.data_ptr())
    engine.sync()
    host = gsa.trace_sparse(gsa.SparseResult(hr.cpu().numpy(), hc.cpu().numpy(), geom, 0, {}), Y, X, sub, -11)
    for budget in ("0", "70000"):  # none, and one 1024 x 256 tile's codes (64 KB)
        knobs("GSA_TRACE_BAND_BUDGET", budget)
        assert engine.trace_sparse_dev(*args, geom, hr.data_ptr(), hc.data_ptr()) == host


def test_score_rejects_out_of_range(engine, golden):
    """gsa_score_dev refuses what its kernels cannot represent, before any launch: scores whose
    unshifted bound reaches 2^30, and SW end-cell keys (score bits + index bits) beyond 63 bits."""
    Y, X = random_pair(3000, 3000, 3)
    huge = np.full((25, 25), 1 << 20, dtype=np.int32)  # 2^20 * 3000 > 2^30
    with pytest.raises(gsa.NwError) as ei:
        engine.score(Y, X, huge, -11, -1, False)
    assert ei.value.stat == gsa.NwStat.errorInvalidValue
    # 100k x 100k: 34 index bits; scores up to 6000 * 1e5 need 30 bits -> 64 > 63
    import torch
    n = 100000
    y = torch.zeros(n + 1, dtype=torch.int32, device="cuda:0")
    big = np.full((25, 25), 6000, dtype=np.int32)
    s = _dev(big)
    with pytest.raises(gsa.NwError) as ei:
        engine.score_dev(y.data_ptr(), n + 1, y.data_ptr(), n + 1, s.data_ptr(), 25, -11, -1, True)
    assert ei.value.stat == gsa.NwStat.errorInvalidValue


def test_score_keeps_fill_error_for_sync(golden):
    """The score kernels keep their error bits in a word of their own: a timed-out fill enqueued
    before a score call is still reported by the caller's next gsa_sync."""
    import oracle
    import torch
    Y, X = random_pair(3000, 2500, 77)
    sub = golden.blosum62
    y, x, s = _dev(Y), _dev(X), _dev(sub)
    args = (y.data_ptr(), len(Y), x.data_ptr(), len(X), s.data_ptr(), 25, -11)
    geom = gsa.sparse_geometry(len(Y), len(X), 128)
    hr = torch.empty(geom.hrowElems, dtype=torch.int32, device="cuda:0")
    hc = torch.empty(geom.hcolElems, dtype=torch.int32, device="cuda:0")
    with gsa.Engine(0) as eng:
        eng.set_watchdog(0)
        eng.fill_sparse_dev(*args, 128, hr.data_ptr(), hc.data_ptr())  # gives up at its first unmet wait
        eng.set_watchdog(1000000)
        r = eng.score_dev(*args, -11, False)
        assert (r["score"], r["i_end"], r["j_end"]) == oracle.score_ag(Y, X, sub, -11, -11, False)
        with pytest.raises(gsa.NwError) as ei:
            eng.sync()
        assert ei.value.stat == gsa.NwStat.errorKernelFailure
        eng.sync()  # cleared
