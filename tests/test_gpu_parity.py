"""GPU parity: the HIP wavefront fills (through the C ABI, libgsa.so) against the oracle.

Bar: bit-exact (integer DP).  Plain family: the whole (R+1)x(C+1) matrix equals
cpu1-st-row's; mlsp family: the whole tileHrowMat/tileHcolMat buffers equal what the
reference's gpu7-9 kernels leave for the same tile geometry (oracle.sparse_headers).  The
reference's own known answers (align_cost, score_hash, trace_hash) are checked end to end.
"""
import numpy as np
import pytest

import gpuseqalign_amd as gsa
import oracle
from tests._data import random_pair, related_pair

pytestmark = pytest.mark.gpu


def _hex(v):
    return "%08x" % v


@pytest.mark.parametrize("idx", range(6))
def test_known_answers_plain(engine, golden, idx):
    case = golden.known["cases"][idx]
    Y, X = golden.pair(case["pair"])
    r = engine.align_full(Y, X, golden.blosum62, golden.known["gapo"])
    assert r.align_cost == case["align_cost"]
    assert _hex(gsa.hash_full(r.score)) == case["score_hash"]
    th, edit = gsa.trace_full(r.score, Y, X)
    assert _hex(th) == case["trace_hash"]
    if "edit_trace" in case:
        assert edit == case["edit_trace"]


@pytest.mark.parametrize("idx", range(6))
def test_known_answers_mlsp(engine, golden, idx):
    case = golden.known["cases"][idx]
    Y, X = golden.pair(case["pair"])
    r = engine.align_sparse(Y, X, golden.blosum62, golden.known["gapo"], tileBx=256)
    assert r.align_cost == case["align_cost"]
    th, edit, cost = gsa.trace_sparse(r, Y, X, golden.blosum62, -11)
    assert _hex(th) == case["trace_hash"] and cost == case["align_cost"]
    if len(Y) * len(X) < 3e7:
        hr, hc, tr, tc, _ = oracle.sparse_headers(Y, X, golden.blosum62, -11, r.geom.tileBy, 256)
        assert np.array_equal(r.hrow, hr) and np.array_equal(r.hcol, hc)


def test_pair_debug_plain(engine, golden):
    """All 173 pairs of resrc/pair_debug.txt (lengths 1..728, tile-edge cases)."""
    for p, Y, X in golden.pairs("pair_debug.txt"):
        r = engine.align_full(Y, X, golden.blosum62, -11)
        S, cost = oracle.fill_full(Y, X, golden.blosum62, -11)
        assert r.align_cost == cost, p
        assert np.array_equal(r.score, S), p


def test_pair_debug_mlsp(engine, golden):
    tBy = gsa.sparse_tile_by()
    for p, Y, X in golden.pairs("pair_debug.txt")[::3]:
        r = engine.align_sparse(Y, X, golden.blosum62, -11, tileBx=64)
        hr, hc, tr, tc, cost = oracle.sparse_headers(Y, X, golden.blosum62, -11, tBy, 64)
        assert r.align_cost == cost, p
        assert np.array_equal(r.hrow, hr), p
        assert np.array_equal(r.hcol, hc), p


EDGES = [1, 2, 62, 63, 64, 65, 126, 127, 252, 253, 255, 256, 257, 505, 1000]


@pytest.mark.parametrize("R", EDGES)
def test_plain_edge_shapes(engine, golden, R):
    for C in (1, 15, 16, 17, 63, 64, 200, 777):
        Y, X = random_pair(R, C, 1000 * R + C)
        r = engine.align_full(Y, X, golden.blosum62, -11)
        S, cost = oracle.fill_full(Y, X, golden.blosum62, -11)
        assert np.array_equal(r.score, S), (R, C)


@pytest.mark.parametrize("tBx", [64, 80, 256, 512])
@pytest.mark.parametrize("R,C", [(1, 1), (63, 64), (252, 256), (253, 257), (700, 300), (300, 1500), (1100, 1029)])
def test_mlsp_shapes(engine, golden, tBx, R, C):
    Y, X = random_pair(R, C, 7 * R + C + tBx)
    r = engine.align_sparse(Y, X, golden.blosum62, -11, tileBx=tBx)
    hr, hc, tr, tc, cost = oracle.sparse_headers(Y, X, golden.blosum62, -11, gsa.sparse_tile_by(), tBx)
    assert (r.trows, r.tcols) == (tr, tc)
    assert np.array_equal(r.hrow, hr)
    assert np.array_equal(r.hcol, hc)
    assert r.align_cost == cost


@pytest.mark.parametrize("name,gapo", [("blosum45", -11), ("blosum80", -1), ("blosum90", -30), ("blosum50", 3)])
def test_other_substitution_and_gaps(engine, golden, name, gapo):
    sub = golden.subst_data.matrix(name)
    Y, X = random_pair(777, 901, 31, alphabet=25)
    r = engine.align_full(Y, X, sub, gapo)
    S, cost = oracle.fill_full(Y, X, sub, gapo)
    assert np.array_equal(r.score, S)
    rs = engine.align_sparse(Y, X, sub, gapo, tileBx=128)
    hr, hc, _, _, _ = oracle.sparse_headers(Y, X, sub, gapo, gsa.sparse_tile_by(), 128)
    assert np.array_equal(rs.hrow, hr) and np.array_equal(rs.hcol, hc)


@pytest.mark.parametrize("ns", [4, 8])
@pytest.mark.parametrize("name,gapo", [("blosum45", -4), ("blosum50", 3), ("blosum90", -30)])
def test_other_substitution_and_gaps_multi_ticket(engine, golden, monkeypatch, ns, name, gapo, knobs):
    """Same over several K-rows tickets (2.5 tile rows): the feed, drain and (ns = 8) mid header
    row carry values of other tables and gap costs, positive included."""
    knobs("GSA_KROW_NS", str(ns))
    sub = golden.subst_data.matrix(name)
    Y, X = random_pair(2500, 2100, 41, alphabet=25)
    rs = engine.align_sparse(Y, X, sub, gapo, tileBx=128)
    hr, hc, _, _, cost = oracle.sparse_headers(Y, X, sub, gapo, gsa.sparse_tile_by(), 128)
    assert np.array_equal(rs.hrow, hr) and np.array_equal(rs.hcol, hc)
    assert rs.align_cost == cost


def test_relaunch_is_deterministic(engine, golden):
    """Back-to-back launches reuse the hand-off buffer under a new epoch tag."""
    Y, X = related_pair(3000, 11)
    a = engine.align_full(Y, X, golden.blosum62, -11).score.copy()
    Y2, X2 = random_pair(1200, 2600, 3)
    engine.align_full(Y2, X2, golden.blosum62, -11)
    b = engine.align_full(Y, X, golden.blosum62, -11).score
    assert np.array_equal(a, b)
    S, _ = oracle.fill_full(Y, X, golden.blosum62, -11)
    assert np.array_equal(a, S)


def test_device_api_on_torch_stream(engine, golden):
    import torch
    Y, X = random_pair(2000, 2500, 77)
    dev = torch.device("cuda:0")
    tY = torch.from_numpy(Y).to(dev)
    tX = torch.from_numpy(X).to(dev)
    tS = torch.from_numpy(golden.blosum62).to(dev)
    out = torch.full((len(Y), len(X)), -7, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream()
    engine.fill_full_dev(tY.data_ptr(), len(Y), tX.data_ptr(), len(X), tS.data_ptr(), 25, -11, out.data_ptr(),
                         s.cuda_stream)
    engine.sync(s.cuda_stream)
    S, _ = oracle.fill_full(Y, X, golden.blosum62, -11)
    assert np.array_equal(out.cpu().numpy(), S)


def test_10k_config_plain_and_mlsp(engine, golden):
    """Config 2 pair (len12124[:10000] x len15390[:10000]) both representations."""
    Y, X = golden.pair("len12124[:10000] len15390[:10000]")
    r = engine.align_full(Y, X, golden.blosum62, -11)
    S, cost = oracle.fill_full(Y, X, golden.blosum62, -11)
    assert np.array_equal(r.score, S)
    rs = engine.align_sparse(Y, X, golden.blosum62, -11, tileBx=256)
    hr, hc, _, _, c2 = oracle.sparse_headers(Y, X, golden.blosum62, -11, gsa.sparse_tile_by(), 256)
    assert np.array_equal(rs.hrow, hr) and np.array_equal(rs.hcol, hc) and rs.align_cost == cost == c2


def test_mlsp_40k_related(engine, golden):
    """Beyond a tile-row count of 150: every header buffer word against the streaming oracle."""
    Y, X = related_pair(40000, 101)
    rs = engine.align_sparse(Y, X, golden.blosum62, -11, tileBx=512)
    hr, hc, _, _, cost = oracle.sparse_headers(Y, X, golden.blosum62, -11, gsa.sparse_tile_by(), 512)
    assert np.array_equal(rs.hrow, hr)
    assert np.array_equal(rs.hcol, hc)
    assert rs.align_cost == cost


@pytest.mark.parametrize("ns", ["1", "2", "3", "4", "6", "8"])
@pytest.mark.parametrize("R,C", [(1, 1), (1, 700), (63, 64), (64, 65), (127, 300), (128, 128), (129, 1029),
                                 (300, 1), (385, 1500), (1100, 2222), (2049, 777)])
def test_full_kernel_shapes(engine, golden, ns, R, C, monkeypatch, knobs):
    """The full-fill kernel (nw_lane.hip, one row per lane) with 1..4, 6, 8 strips per workgroup
    (GSA_LANE_NS, read per launch): every super-strip boundary, ragged last strips, rows beyond
    R, every word."""
    knobs("GSA_FULL_KERNEL", "lane")
    knobs("GSA_LANE_NS", ns)
    Y, X = random_pair(R, C, 3 * R + C)
    r = engine.align_full(Y, X, golden.blosum62, -11)
    S, cost = oracle.fill_full(Y, X, golden.blosum62, -11)
    assert np.array_equal(r.score, S) and r.align_cost == cost


@pytest.mark.parametrize("ns", ["1", "2", "3", "4", "8"])
def test_lane_kernel_wide_pair(engine, golden, ns, monkeypatch, knobs):
    """Columns past the profile ring (512 columns, 1024 from NS = 5) and its guard copies,
    several super-strips."""
    knobs("GSA_FULL_KERNEL", "lane")
    knobs("GSA_LANE_NS", ns)
    Y, X = related_pair(5000, 17)
    r = engine.align_full(Y, X, golden.blosum62, -11)
    S, cost = oracle.fill_full(Y, X, golden.blosum62, -11)
    assert np.array_equal(r.score, S) and r.align_cost == cost



@pytest.mark.parametrize("R,C,off", [(1, 1, 0), (2, 3, 1), (63, 64, 3), (64, 65, 0), (129, 1029, 7), (300, 1, 5),
                                     (385, 1500, 13), (1100, 2222, 1), (2049, 777, 15), (700, 4099, 9)])
def test_full_fill_at_unaligned_base(engine, golden, R, C, off):
    """The full fill into a device buffer that starts 0..15 ints past a 64-byte boundary: every
    matrix word equals the oracle and the words around the matrix stay untouched (the transposed
    stores address rows by a scalar base plus lane offsets; edge blocks store per element)."""
    import torch
    Y, X = random_pair(R, C, 7 * R + C + off)
    dev = torch.device("cuda:0")
    y, x = torch.from_numpy(Y).to(dev), torch.from_numpy(X).to(dev)
    s = torch.from_numpy(golden.blosum62).to(dev)
    n = len(Y) * len(X)
    buf = torch.full((n + 16 + off,), -7, dtype=torch.int32, device=dev)
    engine.fill_full_dev(y.data_ptr(), len(Y), x.data_ptr(), len(X), s.data_ptr(), 25, -11, buf.data_ptr() + 4 * off)
    engine.sync()
    out = buf.cpu().numpy()
    S, _ = oracle.fill_full(Y, X, golden.blosum62, -11)
    assert (out[:off] == -7).all() and (out[off + n:] == -7).all()
    assert np.array_equal(out[off:off + n].reshape(len(Y), len(X)), S)


@pytest.mark.parametrize("R,C,pad,off", [(1, 1, 0, 31), (2, 3, 5, 31), (63, 64, -1, 31), (64, 65, -1, 31),
                                         (129, 1029, -1, 31), (300, 1, -1, 31), (385, 1500, -1, 0),
                                         (1100, 2222, -1, 31), (2049, 777, 33, 17), (700, 4099, -1, 31)])
def test_full_fill_pitched(engine, golden, R, C, pad, off):
    """Pitched device layout (gsa_fill_full_pitched_dev): row pitch gsa_full_pitch (pad -1) or
    adjcols + pad, the matrix `off` ints past a 128-byte boundary.  Every cell equals the oracle;
    the padding columns and the words around the matrix stay untouched."""
    import torch
    Y, X = random_pair(R, C, 5 * R + C + off)
    dev = torch.device("cuda:0")
    y, x = torch.from_numpy(Y).to(dev), torch.from_numpy(X).to(dev)
    s = torch.from_numpy(golden.blosum62).to(dev)
    ld = gsa.full_pitch(len(X)) if pad < 0 else len(X) + pad
    assert ld >= len(X) and (pad >= 0 or ld % 32 == 1)
    n = len(Y) * ld
    buf = torch.full((n + 64 + off,), -7, dtype=torch.int32, device=dev)
    engine.fill_full_dev(y.data_ptr(), len(Y), x.data_ptr(), len(X), s.data_ptr(), 25, -11, buf.data_ptr() + 4 * off,
                         ld=ld)
    engine.sync()
    out = buf.cpu().numpy()
    S, _ = oracle.fill_full(Y, X, golden.blosum62, -11)
    assert (out[:off] == -7).all() and (out[off + n:] == -7).all()
    M = out[off:off + n].reshape(len(Y), ld)
    assert np.array_equal(M[:, :len(X)], S)
    assert (M[:, len(X):] == -7).all()


def test_full_pitch_contract(engine):
    """gsa_full_pitch: the smallest ld >= adjcols with ld = 1 (mod 32); a pitch below adjcols is
    rejected with errorInvalidValue."""
    for ac in (1, 2, 32, 33, 34, 64, 65, 10001, 20001, 20032, 2**31 - 31):
        ld = gsa.full_pitch(ac)
        assert ld >= ac and ld % 32 == 1 and ld - 32 < ac
    assert gsa.full_pitch(2**31 - 30) == 0 and gsa.full_pitch(2**31 - 1) == 0  # past int32: no pitch
    assert gsa.full_base_offset() == 31
    import torch
    dev = torch.device("cuda:0")
    t = torch.zeros(64, dtype=torch.int32, device=dev)
    with pytest.raises(gsa.NwError) as ei:
        engine.fill_full_dev(t.data_ptr(), 4, t.data_ptr(), 4, t.data_ptr(), 1, -11, t.data_ptr(), ld=3)
    assert ei.value.stat == gsa.NwStat.errorInvalidValue


@pytest.mark.parametrize("pair", ["0", "1"])
@pytest.mark.parametrize("ns", ["2", "4", "8"])
def test_full_batch_pitched(engine, golden, ns, pair, monkeypatch, knobs):
    """The one-pass lane fill's batch path (GSA_FULL_KERNEL=lane; batches default to the two-pass
    fill, covered by test_twopass_tables_and_batches) into pitched matrices
    (gsa_fill_full_batch_pitched_dev) and unpadded ones (shard.gpu_batch_align), with and without
    paired stores (GSA_LANE_PAIR; NS != 4 always pairs): every cell of every pair against the oracle."""
    import torch
    from gpuseqalign_amd import shard
    knobs("GSA_FULL_KERNEL", "lane")
    knobs("GSA_LANE_NS", ns)
    knobs("GSA_LANE_PAIR", pair)
    pairs = [random_pair(r, c, 11 * r + c) for r, c in ((700, 900), (1, 5), (1500, 333), (257, 2049), (64, 64))]
    dev = torch.device("cuda:0")
    s = torch.from_numpy(golden.blosum62).to(dev)
    ins = [(torch.from_numpy(Y).to(dev), torch.from_numpy(X).to(dev)) for Y, X in pairs]
    lds = [gsa.full_pitch(len(X)) for _, X in pairs]
    bufs = [torch.full((len(Y) * ld + 64,), -7, dtype=torch.int32, device=dev) for (Y, _), ld in zip(pairs, lds)]
    engine.fill_batch_dev([(y.data_ptr(), len(y), x.data_ptr(), len(x), b.data_ptr() + 4 * 31)
                           for (y, x), b in zip(ins, bufs)], s.data_ptr(), 25, -11, mode="full", lds=lds)
    engine.sync()
    for (Y, X), b, ld in zip(pairs, bufs, lds):
        out = b.cpu().numpy()[31:31 + len(Y) * ld].reshape(len(Y), ld)
        S, _ = oracle.fill_full(Y, X, golden.blosum62, -11)
        assert np.array_equal(out[:, :len(X)], S)
    costs, _ = shard.gpu_batch_align(0, mode="full")(list(range(len(pairs))), pairs, golden.blosum62, -11)
    assert costs == [int(oracle.fill_full(Y, X, golden.blosum62, -11)[1]) for Y, X in pairs]


@pytest.mark.parametrize("kernel", ["lane", "twopass", "fused", "fused_staged"])
@pytest.mark.parametrize("R,C", [(1, 1), (1, 300), (300, 1), (63, 64), (64, 64), (65, 257), (255, 256), (256, 512),
                                 (511, 513), (513, 1024), (1023, 700), (1025, 1029), (2049, 300), (3100, 2222)])
def test_full_fill_kernels(engine, golden, kernel, R, C, monkeypatch, knobs):
    """The full-fill kernels (GSA_FULL_KERNEL, GSA_FULL_FUSED): the one-pass lane fill, the two-pass
    fill in two launches (K-rows pass 1 keeping every 64th row and the 256-column tile header columns,
    then every 64 x 512 tile recomputed by nw_expand.hip) and in one (the fused single-pair kernel;
    its strips store row 64m themselves at these sizes, or hand it to the storer wave as large pairs
    do, GSA_FUSED_STAGED=1): every word, around the 64-row, 256-column and 1024-row tile edges."""
    knobs("GSA_FULL_KERNEL", "lane" if kernel == "lane" else "twopass")
    knobs("GSA_FULL_FUSED", "0" if kernel in ("lane", "twopass") else "1")
    if kernel == "fused_staged":
        knobs("GSA_FUSED_STAGED", "1")
    Y, X = random_pair(R, C, 13 * R + C)
    r = engine.align_full(Y, X, golden.blosum62, -11)
    S, cost = oracle.fill_full(Y, X, golden.blosum62, -11)
    assert np.array_equal(r.score, S) and r.align_cost == cost


@pytest.mark.parametrize("ns", ["4", "8"])
@pytest.mark.parametrize("name,gapo", [("blosum45", -5), ("blosum80", -30), ("blosum62", 3), ("blosum50", -70)])
def test_twopass_tables_and_batches(engine, golden, ns, name, gapo, monkeypatch, knobs):
    """The two-pass fill of a batch in both pass-1 geometries (4 strips: 1024-row tickets, 8 strips:
    2048-row tickets, GSA_KROW_NS) and the streamed expansion (a loader wave staging each task's
    inputs for 7 tile waves), other tables and gap costs (a positive gap included; at gap -70
    s - 2g leaves int8 and pass 1 runs its int16 instance), pitched layout, every word of every pair
    against the oracle, and the words around each matrix untouched."""
    import torch
    knobs("GSA_FULL_KERNEL", "twopass")
    knobs("GSA_KROW_NS", ns)
    knobs("GSA_FULL_FUSED", "0")
    sub = golden.subst_data.matrix(name)
    pairs = [random_pair(r, c, 7 * r + c, alphabet=25) for r, c in ((2100, 900), (1, 5), (700, 2500), (64, 64), (4097, 300))]
    dev = torch.device("cuda:0")
    s = torch.from_numpy(np.ascontiguousarray(sub, dtype=np.int32)).to(dev)
    ins = [(torch.from_numpy(Y).to(dev), torch.from_numpy(X).to(dev)) for Y, X in pairs]
    lds = [gsa.full_pitch(len(X)) for _, X in pairs]
    bufs = [torch.full((len(Y) * ld + 64,), -7, dtype=torch.int32, device=dev) for (Y, _), ld in zip(pairs, lds)]
    engine.fill_batch_dev([(y.data_ptr(), len(y), x.data_ptr(), len(x), b.data_ptr() + 4 * 31)
                           for (y, x), b in zip(ins, bufs)], s.data_ptr(), 25, gapo, mode="full", lds=lds)
    engine.sync()
    for (Y, X), b, ld in zip(pairs, bufs, lds):
        out = b.cpu().numpy()
        M = out[31:31 + len(Y) * ld].reshape(len(Y), ld)
        S, _ = oracle.fill_full(Y, X, sub, gapo)
        assert np.array_equal(M[:, :len(X)], S)
        assert (out[:31] == -7).all() and (out[31 + len(Y) * ld:] == -7).all()


@pytest.mark.parametrize("staged", ["0", "1"])
@pytest.mark.parametrize("name,gapo", [("blosum45", -5), ("blosum62", 3), ("blosum50", -70)])
def test_fused_tables_pitched_repeated(engine, golden, name, gapo, staged, monkeypatch, knobs):
    """The fused single-pair fill (pass-1 tickets and expansion tasks in one launch, hand-off through
    per-strip progress words): other tables and gaps (-70: the int16 instance behind the declining
    int8 one), pitched and unpadded, launched back to back on one stream (a task that ran ahead of
    its strips' words would read the previous launch's rows): every word every time."""
    import torch
    knobs("GSA_FULL_KERNEL", "twopass")
    knobs("GSA_FULL_FUSED", "1")
    knobs("GSA_FUSED_STAGED", staged)
    sub = golden.subst_data.matrix(name)
    dev = torch.device("cuda:0")
    s = torch.from_numpy(np.ascontiguousarray(sub, dtype=np.int32)).to(dev)
    for R, C, pitched in ((3100, 4700, True), (2049, 1537, False)):
        Y, X = random_pair(R, C, 5 * R + C, alphabet=25)
        S, _ = oracle.fill_full(Y, X, sub, gapo)
        y, x = torch.from_numpy(Y).to(dev), torch.from_numpy(X).to(dev)
        ld = gsa.full_pitch(len(X)) if pitched else len(X)
        off = gsa.full_base_offset() if pitched else 0
        n = len(Y) * ld
        bufs = [torch.full((n + 64 + off,), -7, dtype=torch.int32, device=dev) for _ in range(6)]
        for rep in range(2):
            for b in bufs:
                if rep:
                    b.fill_(-7)
                engine.fill_full_dev(y.data_ptr(), len(Y), x.data_ptr(), len(X), s.data_ptr(), 25, gapo,
                                     b.data_ptr() + 4 * off, ld=ld if pitched else None)
            engine.sync()
            for b in bufs:
                out = b.cpu().numpy()
                M = out[off:off + n].reshape(len(Y), ld)
                assert np.array_equal(M[:, :len(X)], S)
                assert (out[:off] == -7).all() and (out[off + n:] == -7).all()


def test_split_batch_single_pair_group(engine, golden, monkeypatch, knobs):
    """a split batch (GSA_FULL_SPLIT=1) whose group A is one pair, with the fused
    single-pair fill left at its default: the groups' passes stay ordered by their events (a fused
    group A recorded none, and group B's pass 1 and expansion then raced it).  Group A: one pair of
    exactly one round of (8, 4) tickets (cu_count x 2048 rows, 100 columns); group B: two pairs of
    20 tickets.  Every word of every pair against the oracle, on two launches."""
    import torch
    knobs("GSA_FULL_KERNEL", "twopass")
    knobs("GSA_FULL_FUSED", None)
    knobs("GSA_KROW_NS", None)
    knobs("GSA_EXPAND_RR", None)
    knobs("GSA_FULL_SPLIT", "1")
    cu = int(engine.cu_count)
    shapes = [(cu * 2048, 100), (40960, 300), (40960, 257)]
    pairs = [random_pair(r, c, 3 * r + c) for r, c in shapes]
    ref = [oracle.fill_full(Y, X, golden.blosum62, -11)[0] for Y, X in pairs]
    dev = torch.device("cuda:0")
    s = torch.from_numpy(golden.blosum62).to(dev)
    ins = [(torch.from_numpy(Y).to(dev), torch.from_numpy(X).to(dev)) for Y, X in pairs]
    bufs = [torch.empty((len(Y) * len(X),), dtype=torch.int32, device=dev) for Y, X in pairs]
    for launch in range(2):
        for b in bufs:
            b.fill_(-7)
        engine.fill_batch_dev([(y.data_ptr(), len(y), x.data_ptr(), len(x), b.data_ptr())
                               for (y, x), b in zip(ins, bufs)], s.data_ptr(), 25, -11, mode="full")
        engine.sync()
        for (Y, X), b, S in zip(pairs, bufs, ref):
            assert np.array_equal(b.cpu().numpy().reshape(len(Y), len(X)), S), launch


@pytest.mark.parametrize("order", ["tuned", "0", "1", "2", "3"])
def test_expansion_orders_repeated(engine, golden, order, monkeypatch, knobs):
    """A batch's expansion task orders (gsa_capi.hip enqueue_full_twopass): by default the first two
    launches on an output buffer run orders 1 and 2 (timed) and later ones the faster; fixed orders
    under GSA_EXPAND_RR (0 pair-major, 1 round-robin, 2 rotated round-robin, 3 shuffled).  Four
    launches back to back on the same buffers (the matrices cleared in between), every word against
    the oracle each time; then a new buffer set restarts the tuning."""
    import torch
    knobs("GSA_FULL_KERNEL", "twopass")
    knobs("GSA_FULL_FUSED", "0")
    if order == "tuned":
        knobs("GSA_EXPAND_RR", None)
    else:
        knobs("GSA_EXPAND_RR", order)
    sub = golden.blosum62
    pairs = [random_pair(r, c, 3 * r + c + 1) for r, c in ((1500, 900), (300, 2500), (2100, 700), (65, 64), (900, 1300))]
    ref = [oracle.fill_full(Y, X, sub, -11)[0] for Y, X in pairs]
    dev = torch.device("cuda:0")
    s = torch.from_numpy(np.ascontiguousarray(sub, dtype=np.int32)).to(dev)
    ins = [(torch.from_numpy(Y).to(dev), torch.from_numpy(X).to(dev)) for Y, X in pairs]
    lds = [gsa.full_pitch(len(X)) for _, X in pairs]
    for buffer_set in range(2):
        bufs = [torch.empty((len(Y) * ld,), dtype=torch.int32, device=dev) for (Y, _), ld in zip(pairs, lds)]
        for launch in range(4):
            for b in bufs:
                b.fill_(-7)
            engine.fill_batch_dev([(y.data_ptr(), len(y), x.data_ptr(), len(x), b.data_ptr())
                                   for (y, x), b in zip(ins, bufs)], s.data_ptr(), 25, -11, mode="full", lds=lds)
            engine.sync()
            for (Y, X), b, ld, S in zip(pairs, bufs, lds, ref):
                M = b.cpu().numpy().reshape(len(Y), ld)
                assert np.array_equal(M[:, :len(X)], S), (buffer_set, launch)


@pytest.mark.parametrize("split", ["tuned", "0", "1"])
def test_full_batch_split(engine, golden, split, monkeypatch, knobs):
    """A full batch whose pass-1 tickets fill one round and part of another, split in two groups
    (GSA_FULL_SPLIT=1: the first round's pairs on the caller's stream, the rest on a high-priority
    stream behind their pass 1, each group with its own pass-1 scratch and expansion order), against
    the same batch in one group (0), and by default (tuned) the first launch untimed in one group,
    one group on the next two launches and two on the two after (gsa_capi.hip enqueue_full), then
    the fastest: every word of every pair equals the oracle on every launch."""
    import torch
    knobs("GSA_FULL_KERNEL", "twopass")
    knobs("GSA_FULL_FUSED", "0")
    if split == "tuned":
        knobs("GSA_FULL_SPLIT", None)
    else:
        knobs("GSA_FULL_SPLIT", split)
    knobs("GSA_KROW_NS", None)
    knobs("GSA_EXPAND_RR", None)
    sub = golden.blosum62
    cu = int(engine.cu_count)
    n = cu + cu // 3  # (8, 4) tickets: 3 per pair of 4100-5100 rows -> 1 round and a part
    rng = np.random.default_rng(31)
    shapes = [(int(rng.integers(4100, 5100)), int(rng.integers(200, 700))) for _ in range(n // 3 + 8)]
    pairs = [random_pair(r, c, 17 * r + c) for r, c in shapes]
    ref = [oracle.fill_full(Y, X, sub, -11)[0] for Y, X in pairs]
    dev = torch.device("cuda:0")
    s = torch.from_numpy(np.ascontiguousarray(sub, dtype=np.int32)).to(dev)
    ins = [(torch.from_numpy(Y).to(dev), torch.from_numpy(X).to(dev)) for Y, X in pairs]
    lds = [gsa.full_pitch(len(X)) for _, X in pairs]
    bufs = [torch.empty((len(Y) * ld,), dtype=torch.int32, device=dev) for (Y, _), ld in zip(pairs, lds)]
    engine.set_full_timing(True)
    try:
        for launch in range(7 if split == "tuned" else 2):
            for b in bufs:
                b.fill_(-7)
            engine.fill_batch_dev([(y.data_ptr(), len(y), x.data_ptr(), len(x), b.data_ptr())
                                   for (y, x), b in zip(ins, bufs)], s.data_ptr(), 25, -11, mode="full", lds=lds)
            engine.sync()
            groups = engine.last_full_timing()["pipelined_groups"]
            if split == "tuned":
                # the first launch untimed (one group), then one group at orders 1 and 2, two groups at
                # orders 1 and 2, then the fastest
                assert groups == (0 if launch < 3 else 2) if launch < 5 else groups in (0, 2), launch
            else:
                assert groups == (2 if split == "1" else 0)
            for (Y, X), b, ld, S in zip(pairs, bufs, lds, ref):
                M = b.cpu().numpy().reshape(len(Y), ld)
                assert np.array_equal(M[:, :len(X)], S), launch
    finally:
        engine.set_full_timing(False)
