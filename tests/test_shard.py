"""Pair sharding (gpuseqalign_amd/shard.py).

CPU: LPT partition properties, the synthetic batch, and the distributed protocol on
world_size 2 over gloo (substitution table broadcast from rank 0, disjoint per-rank results
gathered to every rank, max-over-ranks time).  The per-rank alignment there is the oracle,
injected by the test as the `align_batch` callable: these tests check the sharding and the
collectives, the fills themselves are checked by the GPU test below and test_gpu_parity.py.
"""
import os
import socket

import numpy as np
import pytest

from gpuseqalign_amd import shard
from tests._data import random_pair


def test_lpt_partition_properties():
    rng = np.random.default_rng(5)
    w = rng.integers(1, 1000, size=97).tolist()
    for n in (1, 2, 3, 8):
        parts = shard.lpt_partition(w, n)
        flat = sorted(i for p in parts for i in p)
        assert flat == list(range(len(w)))
        loads = [sum(w[i] for i in p) for p in parts]
        # LPT bound: makespan <= 4/3 OPT, and OPT >= max(mean load, max item)
        opt_lb = max(sum(w) / n, max(w))
        assert max(loads) <= 4 / 3 * opt_lb + 1e-9
        assert parts == shard.lpt_partition(w, n)  # deterministic
    assert shard.lpt_partition([3, 3], 4) == [[0], [1], [], []]
    with pytest.raises(ValueError):
        shard.lpt_partition([1], 0)


def test_synthetic_batch_shape():
    b = shard.synthetic_batch(6, 50, 80, seed0=1000)
    assert len(b) == 6
    for y, x in b:
        assert y[0] == 0 and x[0] == 0
        assert 50 <= len(y) - 1 <= 80 and 50 <= len(x) - 1 <= 80
        assert y.dtype == np.int32 and y[1:].max() < 20
    b2 = shard.synthetic_batch(6, 50, 80, seed0=1000)
    assert all(np.array_equal(a[0], c[0]) and np.array_equal(a[1], c[1]) for a, c in zip(b, b2))


def _oracle_batch(indices, pairs, subst, gapo):
    import oracle
    costs = []
    for i in indices:
        _, c = oracle.fill_full(pairs[i][0], pairs[i][1], subst, gapo)
        costs.append(int(c))
    return costs, 0.001 * (len(indices) + 1)


def _pairs():
    return [random_pair(r, c, 17 * r + c) for r, c in [(40, 50), (120, 30), (7, 9), (64, 64), (200, 150), (1, 5),
                                                       (90, 91), (33, 256), (150, 12)]]


def _worker(rank, world, port, subst, gapo, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rep = shard.shard_align(_pairs(), subst if rank == 0 else None, gapo, _oracle_batch)
        q.put((rank, [(r.index, r.align_cost, r.cells, r.rank) for r in rep.results], rep.elapsed_s, rep.world))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_gloo_world2(golden):
    import torch.multiprocessing as mp
    subst = golden.blosum62
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, subst, -11, q)) for r in range(2)]
    for p in procs:
        p.start()
    outs = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    import oracle
    pairs = _pairs()
    expect = [int(oracle.fill_full(y, x, subst, -11)[1]) for y, x in pairs]
    weights = [(len(y) - 1) * (len(x) - 1) for y, x in pairs]
    parts = shard.lpt_partition(weights, 2)
    for rank, res, secs, world in outs:
        assert world == 2
        assert [r[1] for r in res] == expect          # gathered costs, in pair order, on every rank
        assert [r[2] for r in res] == weights
        for i, _, _, owner in res:
            assert i in parts[owner]                  # each pair on its LPT rank
        assert secs == pytest.approx(0.001 * (max(len(p) for p in parts) + 1))  # max over ranks


def test_shard_single_process_no_dist(golden):
    rep = shard.shard_align(_pairs(), golden.blosum62, -11, _oracle_batch)
    assert rep.world == 1 and len(rep.results) == 9 and all(r.rank == 0 for r in rep.results)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["full", "sparse"])
def test_gpu_batch_matches_oracle(golden, mode):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU visible")
    import oracle
    pairs = _pairs() + shard.synthetic_batch(5, 900, 1500, seed0=2000)
    expect = [int(oracle.fill_full(y, x, golden.blosum62, -11)[1]) for y, x in pairs]
    # one launch for the whole batch, and a budget that forces several launches
    for budget in (None, 3 * 1024 * 1024):
        rep = shard.shard_align(pairs, golden.blosum62, -11,
                                shard.gpu_batch_align(0, mode=mode, tileBx=128, out_budget_bytes=budget))
        assert [r.align_cost for r in rep.results] == expect
        assert rep.elapsed_s > 0 and rep.gcups > 0


@pytest.mark.gpu
@pytest.mark.parametrize("order", ["round-robin", "pair"])
@pytest.mark.parametrize("mode", ["full", "sparse"])
def test_batched_launch_equals_single_fills(engine, golden, mode, order, monkeypatch):
    """Every output word of a batched launch equals the single-pair fill of the same pair, with
    the tickets scheduled round-robin over the pairs (default) or pair-major (GSA_BATCH_ORDER)."""
    monkeypatch.setenv("GSA_BATCH_ORDER", order)
    import torch
    import gpuseqalign_amd as gsa
    # + pairs of 2-5 tickets (256-row super-strips), so the schedule interleaves their chains
    pairs = _pairs() + [random_pair(r, c, 5 * r + c) for r, c in [(700, 300), (1030, 200), (600, 900), (300, 77)]]
    dev = torch.device("cuda:0")
    ts = torch.from_numpy(golden.blosum62).to(dev)
    ins = [(torch.from_numpy(y).to(dev), torch.from_numpy(x).to(dev)) for y, x in pairs]
    outs, descs = [], []
    for y, x in ins:
        if mode == "sparse":
            g = gsa.sparse_geometry(len(y), len(x), 64)
            o = (torch.full((g.hrowElems,), -7, dtype=torch.int32, device=dev),
                 torch.full((g.hcolElems,), -7, dtype=torch.int32, device=dev))
            descs.append((y.data_ptr(), len(y), x.data_ptr(), len(x), (o[0].data_ptr(), o[1].data_ptr())))
        else:
            o = (torch.full((len(y) * len(x),), -7, dtype=torch.int32, device=dev),)
            descs.append((y.data_ptr(), len(y), x.data_ptr(), len(x), o[0].data_ptr()))
        outs.append(o)
    engine.fill_batch_dev(descs, ts.data_ptr(), 25, -11, mode=mode, tileBx=64)
    engine.sync()
    for (y, x), o in zip(pairs, outs):
        if mode == "sparse":
            r = engine.align_sparse(y, x, golden.blosum62, -11, tileBx=64)
            assert np.array_equal(o[0].cpu().numpy(), r.hrow) and np.array_equal(o[1].cpu().numpy(), r.hcol)
        else:
            r = engine.align_full(y, x, golden.blosum62, -11)
            assert np.array_equal(o[0].cpu().numpy().reshape(len(y), len(x)), r.score)
