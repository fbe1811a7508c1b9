"""Sparse traceback on the device (gsa_trace_sparse_dev, nw_trace_dev.hip)
against the host NwTrace2_Sparse restatement (gsa_trace_sparse, itself pinned to the
reference's known trace hashes by test_capi / test_oracle_golden) and the oracle's trace."""
import numpy as np
import pytest

import gpuseqalign_amd as gsa
from tests._data import random_pair, related_pair

pytestmark = pytest.mark.gpu


def _dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.int32)).to("cuda:0")


def _both(engine, Y, X, sub, gapo, tBx):
    """Device fill, then the device trace (headers stay in HBM) and the host trace."""
    import torch
    geom = gsa.sparse_geometry(len(Y), len(X), tBx)
    y, x, s = _dev(Y), _dev(X), _dev(sub)
    hr = torch.empty(geom.hrowElems, dtype=torch.int32, device="cuda:0")
    hc = torch.empty(geom.hcolElems, dtype=torch.int32, device="cuda:0")
    ss = int(round(np.sqrt(np.asarray(sub).size)))
    args = (y.data_ptr(), len(Y), x.data_ptr(), len(X), s.data_ptr(), ss, gapo)
    engine.fill_sparse_dev(*args, tBx, hr.data_ptr(), hc.data_ptr())
    engine.sync()
    dev = engine.trace_sparse_dev(*args, geom, hr.data_ptr(), hc.data_ptr())
    res = gsa.SparseResult(hr.cpu().numpy(), hc.cpu().numpy(), geom, 0, {})
    host = gsa.trace_sparse(res, Y, X, sub, gapo)
    return dev, host


@pytest.mark.parametrize("R,C,tBx,related", [(0, 0, 64, False), (0, 37, 64, False), (41, 0, 64, False),
                                             (1, 1, 64, False), (700, 900, 64, True), (1024, 1024, 64, True),
                                             (1023, 2048, 128, True), (2049, 777, 80, False),
                                             (3000, 3000, 256, True), (2500, 2600, 512, True),
                                             (2500, 2600, 1024, True), (1500, 5000, 4096, False)])
def test_device_trace_equals_host(engine, golden, R, C, tBx, related):
    if related:
        Y, X = related_pair(R, R + C)
        X = X[:C + 1] if len(X) > C + 1 else X
    else:
        Y, X = random_pair(R, C, 5 * R + C + 1)
    dev, host = _both(engine, Y, X, golden.blosum62, -11, tBx)
    assert dev == host


def test_device_trace_pair_debug(engine, golden):
    """Every pair of the reference's pair_debug.txt: hashes and edit strings as the host trace,
    costs as the oracle."""
    import oracle
    for p, Y, X in golden.pairs("pair_debug.txt"):
        dev, host = _both(engine, Y, X, golden.blosum62, -11, 64)
        assert dev == host, p
        assert dev[2] == oracle.fill_full(Y, X, golden.blosum62, -11)[1]


def test_device_trace_known_answer(engine, golden):
    """len31 x len32 and len728 x len728: the reference's trace hashes and edit strings."""
    for line, th, edit in [("len31 len32", 0x5e67e0b4, "11X1=19X1D"), ("len728 len728", 0x7c52dee5, "728=")]:
        Y, X = golden.pair(line)
        dev, _ = _both(engine, Y, X, golden.blosum62, -11, 64)
        assert dev[0] == th and dev[1] == edit, (line, dev)


def test_device_trace_100k(engine, golden):
    """BASELINE configs[2]: 100k x 100k related pair; device walk equals the host walk."""
    import time
    from gpuseqalign_amd import formats as F
    X = F.synthetic_seq(100000, 100)
    Y = F.mutate_seq(X, 101)
    t0 = time.perf_counter()
    dev, host = _both(engine, Y, X, golden.blosum62, -11, 256)
    assert dev == host
    assert len(dev[1]) > 1000  # a non-trivial edit path


@pytest.mark.parametrize("band", ["0", "16", "300"])
@pytest.mark.parametrize("R,C,tBx,related", [(3000, 3000, 64, False), (2500, 4100, 128, True), (4100, 1700, 64, False)])
def test_device_trace_band(engine, golden, monkeypatch, band, R, C, tBx, related):
    """Tiles precomputed around the diagonal (GSA_TRACE_BAND columns) and tiles the walk finds
    outside the band (recomputed on entry) give the host walk: no band, a band narrower than a
    tile (random pairs leave it), and a wider one."""
    monkeypatch.setenv("GSA_TRACE_BAND", band)
    if related:
        Y, X = related_pair(R, R + C)
        X = X[:C + 1] if len(X) > C + 1 else X
    else:
        Y, X = random_pair(R, C, 7 * R + C)
    dev, host = _both(engine, Y, X, golden.blosum62, -11, tBx)
    assert dev == host


@pytest.mark.parametrize("name,gapo", [("blosum45", -4), ("blosum50", 3), ("blosum90", -30)])
def test_device_trace_other_tables(engine, golden, name, gapo):
    """Other substitution tables and gap costs (positive included): the band precompute and the
    walk re-derive each move from the recurrence with the caller's table and gap."""
    sub = golden.subst_data.matrix(name)
    Y, X = random_pair(2300, 1900, 5, alphabet=25)
    import oracle
    dev, host = _both(engine, Y, X, sub, gapo, 128)
    assert dev == host
    assert dev[2] == oracle.fill_full(Y, X, sub, gapo)[1]
