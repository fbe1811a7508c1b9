"""Error path of the persistent fills (include/gsa.h: gsa_sync, gsa_set_watchdog).

A hand-off wait that sees no progress for the watchdog's limit gives up and sets the context's
error word.  The word is sticky: a time-out in any launch since the last gsa_sync makes that
sync fail (launches enqueued behind it give up at once), and the sync clears it, so the next
fill on the same context is correct.  The watchdog is forced to 0 (give up at the first unmet
poll) to provoke the time-out; the reference maps such a failure to errorKernelFailure
(run_types.hpp:12-24)."""
import numpy as np
import pytest

import gpuseqalign_amd as gsa
from tests._data import random_pair

pytestmark = pytest.mark.gpu


def _dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.int32)).to("cuda:0")


@pytest.mark.parametrize("mode", ["full", "sparse"])
def test_watchdog_timeout_is_sticky_and_clears(golden, mode):
    import torch
    import oracle
    Y, X = random_pair(3000, 2500, 77)
    sub = golden.blosum62
    y, x, s = _dev(Y), _dev(X), _dev(sub)
    args = (y.data_ptr(), len(Y), x.data_ptr(), len(X), s.data_ptr(), 25, -11)
    with gsa.Engine(0) as eng:
        if mode == "full":
            out = torch.empty(len(Y) * len(X), dtype=torch.int32, device="cuda:0")
            fill = lambda: eng.fill_full_dev(*args, out.data_ptr())
        else:
            geom = gsa.sparse_geometry(len(Y), len(X), 128)
            hr = torch.empty(geom.hrowElems, dtype=torch.int32, device="cuda:0")
            hc = torch.empty(geom.hcolElems, dtype=torch.int32, device="cuda:0")
            fill = lambda: eng.fill_sparse_dev(*args, 128, hr.data_ptr(), hc.data_ptr())
        # launch 1 times out (watchdog 0: the first ticket waiting on another gives up), launch 2
        # is healthy but enqueued behind it before any sync: the sync must still report launch 1
        eng.set_watchdog(0)
        fill()
        eng.set_watchdog(1000000)
        fill()
        with pytest.raises(gsa.NwError) as ei:
            eng.sync()
        assert ei.value.stat == gsa.NwStat.errorKernelFailure
        # cleared by that sync: the same context fills correctly again
        fill()
        eng.sync()
        if mode == "full":
            S, cost = oracle.fill_full(Y, X, sub, -11)
            assert np.array_equal(out.cpu().numpy().reshape(S.shape), S)
        else:
            hrow, hcol, _, _, cost = oracle.sparse_headers(Y, X, sub, -11, gsa.sparse_tile_by(), 128)
            assert np.array_equal(hr.cpu().numpy(), hrow) and np.array_equal(hc.cpu().numpy(), hcol)


def test_watchdog_rejects_bad_values():
    with gsa.Engine(0) as eng:
        with pytest.raises(gsa.NwError):
            eng.set_watchdog(-1)


def test_mem_stats_after_fill(engine, golden):
    """Peak-alloc accounting (updateNwAlgPeakMemUsage, nwalign_shared.cpp:5-25)."""
    import torch
    Y, X = random_pair(1500, 1700, 5)
    y, x, s = _dev(Y), _dev(X), _dev(golden.blosum62)
    engine.reset_mem_stats()
    assert all(v == 0 for v in engine.mem_stats().values())
    geom = gsa.sparse_geometry(len(Y), len(X), 256)
    hr = torch.empty(geom.hrowElems, dtype=torch.int32, device="cuda:0")
    hc = torch.empty(geom.hcolElems, dtype=torch.int32, device="cuda:0")
    engine.fill_sparse_dev(y.data_ptr(), len(Y), x.data_ptr(), len(X), s.data_ptr(), 25, -11, 256, hr.data_ptr(),
                           hc.data_ptr())
    engine.sync()
    m = engine.mem_stats()
    assert m["shmem_peak_allocs"] > 0 and m["regmem_peak_allocs"] > 0 and m["glmem_peak_allocs"] > 0
    assert m["locmem_peak_allocs"] >= 0
