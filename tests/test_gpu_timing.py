"""The full fill's timing aid (gsa_set_full_timing / gsa_last_full_timing): pass times from HIP
events and pass 2's effective clock from per-workgroup s_memtime / s_memrealtime stamps; the
stamps must not change a result (every cell against the oracle)."""
import numpy as np
import pytest

import gpuseqalign_amd as gsa
import oracle
from tests._data import random_pair


@pytest.mark.gpu
def test_full_timing_two_launches(engine, golden, monkeypatch):
    import torch
    monkeypatch.setenv("GSA_FULL_FUSED", "0")
    pairs = [random_pair(r, c, 7 * r + c) for r, c in ((2100, 1900), (700, 3000))]
    dev = torch.device("cuda:0")
    s = torch.from_numpy(golden.blosum62).to(dev)
    ins = [(torch.from_numpy(Y).to(dev), torch.from_numpy(X).to(dev)) for Y, X in pairs]
    bufs = [torch.full((len(Y) * len(X),), -7, dtype=torch.int32, device=dev) for Y, X in pairs]
    with pytest.raises(gsa.NwError):
        engine.last_full_timing()  # nothing timed yet
    engine.set_full_timing(True)
    try:
        engine.fill_batch_dev([(y.data_ptr(), len(y), x.data_ptr(), len(x), b.data_ptr())
                               for (y, x), b in zip(ins, bufs)], s.data_ptr(), 25, -11, mode="full")
        t = engine.last_full_timing()
    finally:
        engine.set_full_timing(False)
    engine.sync()
    assert not t["fused"] and t["pass1_ms"] > 0 and t["pass2_ms"] > 0
    assert t["clock_workgroups"] > 0 and 0.3 < t["clock_ghz_median"] < 3.5 and 0.3 < t["clock_ghz_mean"] < 3.5
    for (Y, X), b in zip(pairs, bufs):
        S, _ = oracle.fill_full(Y, X, golden.blosum62, -11)
        assert np.array_equal(b.cpu().numpy().reshape(len(Y), len(X)), S)


@pytest.mark.gpu
def test_full_timing_fused(engine, golden, monkeypatch):
    import torch
    monkeypatch.setenv("GSA_FULL_FUSED", "1")
    Y, X = random_pair(1500, 1300, 5)
    dev = torch.device("cuda:0")
    s = torch.from_numpy(golden.blosum62).to(dev)
    y, x = torch.from_numpy(Y).to(dev), torch.from_numpy(X).to(dev)
    b = torch.empty(len(Y) * len(X), dtype=torch.int32, device=dev)
    engine.set_full_timing(True)
    try:
        engine.fill_full_dev(y.data_ptr(), len(Y), x.data_ptr(), len(X), s.data_ptr(), 25, -11, b.data_ptr())
        t = engine.last_full_timing()
    finally:
        engine.set_full_timing(False)
    assert t["fused"] and t["pass1_ms"] is None and t["pass2_ms"] > 0 and t["clock_ghz_median"] is None
    S, _ = oracle.fill_full(Y, X, golden.blosum62, -11)
    assert np.array_equal(b.cpu().numpy().reshape(len(Y), len(X)), S)
