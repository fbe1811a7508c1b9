"""Size-scale parity against committed oracle goldens (tools/make_goldens.py; the oracle ran in
the build container, so the GPU box needs neither the oracle nor the reference):

  * BASELINE configs[2] -- the 100k x 100k related pair (seeds 100/101) and the unrelated pair
    (seeds 102/103): HIP sparse fill -> align_cost, every tile-header word (sha256 over
    tileHrowMat + tileHcolMat), and the device Trace2 walk (nwtrace2_sparse.cpp:102-257): trace
    hash and edit string (sha256);
  * BASELINE configs[3] -- all 512 pairs of 18-22k (shard.synthetic_batch, seeds 1000+k) in one
    batched launch: every align_cost against the cpu1 streaming restatement; every header word
    of all 512 pairs by the device checker (tile consistency, gsa_check_sparse_dev), and the
    headers of 16 of them (sha256) against the oracle's, on the batch's 8-strip geometry and on
    the 4-strip one.  The reference itself compares headers only along the trace path
    (nwtrace2_sparse.cpp:263-340, the constant-index quirk at :293).
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


def _load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def _config3(name):
    if name == "related":
        X = F.synthetic_seq(100000, 100)
        return F.mutate_seq(X, 101), X
    return F.synthetic_seq(100000, 102), F.synthetic_seq(100000, 103)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("name", ["related", "unrelated"])
def test_config3_100k_matches_golden(engine, golden, name):
    import torch
    gold = _load("config3_100k.json")["pairs"][name]
    Y, X = _config3(name)
    assert hashlib.sha256(Y.tobytes()).hexdigest() == gold["seqY_sha256"]
    assert hashlib.sha256(X.tobytes()).hexdigest() == gold["seqX_sha256"]
    sub = golden.blosum62
    tBx = 256
    geom = gsa.sparse_geometry(len(Y), len(X), tBx)
    dev = torch.device("cuda:0")
    y, x, s = (torch.from_numpy(np.ascontiguousarray(a, dtype=np.int32)).to(dev) for a in (Y, X, sub))
    hr = torch.empty(geom.hrowElems, dtype=torch.int32, device=dev)
    hc = torch.empty(geom.hcolElems, dtype=torch.int32, device=dev)
    args = (y.data_ptr(), len(Y), x.data_ptr(), len(X), s.data_ptr(), 25, -11)
    engine.fill_sparse_dev(*args, tBx, hr.data_ptr(), hc.data_ptr())
    engine.sync()
    key = "%dx%d" % (geom.tileHcolLen - 1, tBx)
    hrn, hcn = hr.cpu().numpy(), hc.cpu().numpy()
    res = gsa.SparseResult(hrn, hcn, geom, 0, {})
    assert gsa.sparse_align_cost(res, Y, X, sub, -11) == gold["align_cost"]
    if key in gold["headers"]:
        h = hashlib.sha256()
        h.update(hrn.tobytes())
        h.update(hcn.tobytes())
        assert h.hexdigest() == gold["headers"][key]["sha256"], "tile headers differ from the oracle's"
    th, edit, cost = engine.trace_sparse_dev(*args, geom, hr.data_ptr(), hc.data_ptr())
    assert cost == gold["align_cost"]
    assert "%08x" % th == gold["trace_hash"]
    assert len(edit) == gold["edit_trace_len"] and edit.startswith(gold["edit_trace_head"])
    assert hashlib.sha256(edit.encode()).hexdigest() == gold["edit_trace_sha256"]


@pytest.mark.timeout(600)
@pytest.mark.parametrize("tBx", [256, 512])
def test_config4_512_pairs_match_golden(golden, tBx):
    """The configs[3] batch at its real size on one GPU: 512 pairs, one persistent launch."""
    import torch
    from gpuseqalign_amd import shard
    if not torch.cuda.is_available():
        pytest.skip("no GPU visible")
    gold = _load("config4_pairs.json")
    n = gold["n_pairs"]
    pairs = shard.synthetic_batch(n, 18000, 22000, seed0=1000)
    assert [len(y) - 1 for y, _ in pairs] == gold["R"] and [len(x) - 1 for _, x in pairs] == gold["C"]
    run = shard.gpu_batch_align(0, mode="sparse", tileBx=tBx, repeats=1, warmup=1)
    costs, secs = run(list(range(n)), pairs, golden.blosum62, -11)
    bad = [k for k in range(n) if costs[k] != gold["align_cost"][k]]
    assert not bad, ("pairs differing from the oracle", bad[:10], len(bad))
    assert secs > 0


@pytest.mark.timeout(600)
@pytest.mark.parametrize("ns", ["batch-default", "4"])
def test_config4_headers_at_size(engine, golden, monkeypatch, ns, knobs):
    """configs[3] at full size, header by header: one persistent launch over all 512 pairs (the
    batch default is 8 strips per workgroup, two tile rows per ticket), then every pair's
    tile headers through the device checker, and 16 pairs' headers against the oracle."""
    import torch
    from gpuseqalign_amd import shard
    if ns != "batch-default":
        knobs("GSA_KROW_NS", ns)
    gold = _load("config4_pairs.json")
    hd = gold["headers"]
    tBx = hd["tileBx"]
    assert hd["tileBy"] == gsa.sparse_tile_by()
    n = gold["n_pairs"]
    pairs = shard.synthetic_batch(n, 18000, 22000, seed0=1000)
    dev = torch.device("cuda:0")
    sub = golden.blosum62
    ts = torch.from_numpy(sub).to(dev)
    ins, outs, geoms = [], [], []
    for Y, X in pairs:
        g = gsa.sparse_geometry(len(Y), len(X), tBx)
        y, x = torch.from_numpy(Y).to(dev), torch.from_numpy(X).to(dev)
        hr = torch.full((g.hrowElems,), -7, dtype=torch.int32, device=dev)  # poison: every word must be written
        hc = torch.full((g.hcolElems,), -7, dtype=torch.int32, device=dev)
        ins.append((y, x))
        outs.append((hr, hc))
        geoms.append(g)
    engine.fill_batch_dev([(y.data_ptr(), len(y), x.data_ptr(), len(x), (hr.data_ptr(), hc.data_ptr()))
                           for (y, x), (hr, hc) in zip(ins, outs)], ts.data_ptr(), 25, -11, mode="sparse", tileBx=tBx)
    engine.sync()
    bad = []
    for k in range(n):
        (y, x), (hr, hc), g = ins[k], outs[k], geoms[k]
        r = engine.check_sparse_dev(y.data_ptr(), len(y), x.data_ptr(), len(x), ts.data_ptr(), 25, -11, g,
                                    hr.data_ptr(), hc.data_ptr())
        # every header word is compared at least once (nw_check.hip), corners twice
        if r["mismatches"] != 0 or r["checked"] < g.hrowElems + g.hcolElems:
            bad.append((k, r))
    assert not bad, ("pairs whose headers fail the device check", bad[:5], len(bad))
    for k, want in zip(hd["pairs"], hd["sha256"]):
        h = hashlib.sha256()
        h.update(outs[k][0].cpu().numpy().tobytes())
        h.update(outs[k][1].cpu().numpy().tobytes())
        assert h.hexdigest() == want, ("headers differ from the oracle's", k)
