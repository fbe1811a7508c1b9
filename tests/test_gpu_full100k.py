"""The north star's own configuration: the config-3 100k x 100k NW-LG pair filled as a FULL int32
score matrix (9.99e9 cells, 40 GB) in HBM, unpadded (gsa_fill_full_dev, the reference's nw.score
layout) and pitched (gsa_fill_full_pitched_dev), then checked three ways that do not need the
matrix on the host:

  * align_cost = the last cell, against the oracle golden (tests/golden/config3_100k.json);
  * NwHash1_Plain over every cell (src/nwtrace1_plain.cpp:133-154), gsa_hash_full_dev, against the
    golden score_hash the oracle's cpu1-st-row fill produced;
  * every cell against the recurrence (gsa_check_full_dev / _pitched_dev: 0 mismatches);
  * NwTrace1_Plain (src/nwtrace1_plain.cpp:6-131) over the device matrix, gsa_trace_full_dev:
    trace hash and edit string (sha256) against the golden Trace2 walk of the same pair (the
    two walks take the same path: same tie-break over the same matrix values).

The reference itself cannot hold this matrix (int indices, src/math.hpp:5).  Smaller cases pin
gsa_hash_full_dev / gsa_trace_full_dev to the host consumers on pitched and edge shapes.
"""
import hashlib
import json
import os

import numpy as np
import pytest

import gpuseqalign_amd as gsa
from gpuseqalign_amd import formats as F
from tests._data import GOLDEN

pytestmark = pytest.mark.gpu


def _gold(name):
    with open(os.path.join(GOLDEN, "config3_100k.json")) as f:
        return json.load(f)["pairs"][name]


def _pair(name):
    if name == "related":
        X = F.synthetic_seq(100000, 100)
        return F.mutate_seq(X, 101), X
    return F.synthetic_seq(100000, 102), F.synthetic_seq(100000, 103)


@pytest.fixture(scope="module")
def big():
    """One 40 GB device buffer shared by the 100k cases (freed at module end)."""
    import torch
    n = 100001 * 100001 + 256
    buf = torch.empty(n, dtype=torch.int32, device="cuda:0")
    yield buf
    del buf
    torch.cuda.empty_cache()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("name,layout", [("related", "pitched"), ("unrelated", "unpadded")])
def test_full_100k_matrix_matches_golden(engine, golden, big, name, layout):
    import torch
    gold = _gold(name)
    Y, X = _pair(name)
    assert hashlib.sha256(Y.tobytes()).hexdigest() == gold["seqY_sha256"]
    assert hashlib.sha256(X.tobytes()).hexdigest() == gold["seqX_sha256"]
    dev = torch.device("cuda:0")
    y, x, s = (torch.from_numpy(np.ascontiguousarray(a, dtype=np.int32)).to(dev) for a in (Y, X, golden.blosum62))
    R1, C1 = len(Y), len(X)
    if layout == "pitched":
        ld = gsa.full_pitch(C1)
        base = big.data_ptr() + 4 * gsa.full_base_offset()
        assert (base + 4 * ld) % 128 == 0  # cell (1, 0) on a 128-byte boundary
    else:
        ld = C1
        base = big.data_ptr()
    assert (R1 - 1) * ld + C1 <= big.numel() - 64
    big[:1024].fill_(0x5a5a5a5a)  # (stale words from the other case must not matter)
    engine.fill_full_dev(y.data_ptr(), R1, x.data_ptr(), C1, s.data_ptr(), 25, -11, base,
                         ld=ld if layout == "pitched" else None)
    engine.sync()
    off = (base - big.data_ptr()) // 4
    cost = int(big[off + (R1 - 1) * ld + C1 - 1].item())
    assert cost == gold["align_cost"]
    chk = engine.check_full_dev(y.data_ptr(), R1, x.data_ptr(), C1, s.data_ptr(), 25, -11, base,
                                ld=ld if layout == "pitched" else None)
    assert chk["mismatches"] == 0 and chk["checked"] == R1 * C1, chk
    th, edit, tcost = engine.trace_full_dev(y.data_ptr(), R1, x.data_ptr(), C1, base, ld=ld)
    assert tcost == gold["align_cost"]
    assert "%08x" % th == gold["trace_hash"]
    assert len(edit) == gold["edit_trace_len"]
    assert hashlib.sha256(edit.encode()).hexdigest() == gold["edit_trace_sha256"]
    assert "%08x" % engine.hash_full_dev(base, R1, C1, ld=ld) == gold["score_hash"]


@pytest.mark.parametrize("R,C,pad", [(1, 1, 0), (1, 300, 5), (300, 1, 3), (700, 900, 0), (700, 900, 19),
                                     (2049, 1500, 7), (64, 2300, 0)])
def test_device_matrix_consumers_equal_host(engine, golden, R, C, pad):
    """gsa_hash_full_dev / gsa_trace_full_dev on a device matrix (row pitch C + pad) equal the
    host consumers (gsa_hash_full / gsa_trace_full) of the same matrix; the trace's block fetches
    cross block edges at 2049 rows and 2300 columns."""
    import torch
    rng = np.random.default_rng(R * 7919 + C)
    Y = np.concatenate([[0], rng.integers(0, 25, R - 1)]).astype(np.int32)
    X = np.concatenate([[0], rng.integers(0, 25, C - 1)]).astype(np.int32)
    dev = torch.device("cuda:0")
    y, x, s = (torch.from_numpy(np.ascontiguousarray(a, dtype=np.int32)).to(dev) for a in (Y, X, golden.blosum62))
    ld = C + pad
    buf = torch.full((R * ld + 8,), 0x7b7b7b7b, dtype=torch.int32, device=dev)
    engine.fill_full_dev(y.data_ptr(), R, x.data_ptr(), C, s.data_ptr(), 25, -11, buf.data_ptr(),
                         ld=ld if pad else None)
    engine.sync()
    host = buf[:R * ld].cpu().numpy().reshape(R, ld)[:, :C].copy()
    assert engine.hash_full_dev(buf.data_ptr(), R, C, ld=ld) == gsa.hash_full(host)
    th, edit = gsa.trace_full(host, Y, X)
    dth, dedit, dcost = engine.trace_full_dev(y.data_ptr(), R, x.data_ptr(), C, buf.data_ptr(), ld=ld)
    assert (dth, dedit, dcost) == (th, edit, int(host[-1, -1]))
    chk = engine.check_full_dev(y.data_ptr(), R, x.data_ptr(), C, s.data_ptr(), 25, -11, buf.data_ptr(),
                                ld=ld if pad else None)
    assert chk["mismatches"] == 0 and chk["checked"] == R * C


def test_pitched_check_catches_a_corrupted_cell(engine, golden):
    import torch
    R, C, ld = 500, 700, 733
    rng = np.random.default_rng(5)
    Y = np.concatenate([[0], rng.integers(0, 25, R - 1)]).astype(np.int32)
    X = np.concatenate([[0], rng.integers(0, 25, C - 1)]).astype(np.int32)
    dev = torch.device("cuda:0")
    y, x, s = (torch.from_numpy(np.ascontiguousarray(a, dtype=np.int32)).to(dev) for a in (Y, X, golden.blosum62))
    buf = torch.zeros(R * ld + 8, dtype=torch.int32, device=dev)
    engine.fill_full_dev(y.data_ptr(), R, x.data_ptr(), C, s.data_ptr(), 25, -11, buf.data_ptr(), ld=ld)
    engine.sync()
    buf[321 * ld + 456] += 1
    chk = engine.check_full_dev(y.data_ptr(), R, x.data_ptr(), C, s.data_ptr(), 25, -11, buf.data_ptr(), ld=ld)
    assert chk["mismatches"] >= 1 and chk["first"] == 321 * C + 456
