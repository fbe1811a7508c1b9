"""Score-only NW / SW with linear or affine gaps on the GPU (gsa_score, nw_scan.hip; BASELINE
configs[4]) against the CPU restatement oracle/score_oracle.c (parity
unpinned by the reference, which has no such mode; the oracle is pinned by
tests/test_score_oracle.py)."""
import numpy as np
import pytest

import gpuseqalign_amd as gsa
from tests._data import random_pair, related_pair

pytestmark = pytest.mark.gpu

MODES = [(-11, -11, False), (-11, -1, False), (-5, -2, False), (-11, -11, True), (-11, -1, True), (-5, -2, True)]


@pytest.mark.parametrize("R,C", [(1, 1), (1, 300), (300, 1), (63, 64), (64, 65), (65, 63), (130, 700), (700, 130),
                                 (1000, 1500)])
@pytest.mark.parametrize("go,ge,local", MODES)
def test_score_matches_oracle(engine, golden, R, C, go, ge, local):
    import oracle
    Y, X = random_pair(R, C, 3 * R + C)
    r = engine.score(Y, X, golden.blosum62, go, ge, local)
    assert (r["score"], r["i_end"], r["j_end"]) == oracle.score_ag(Y, X, golden.blosum62, go, ge, local)


@pytest.mark.parametrize("n", [200, 2000, 4097])
@pytest.mark.parametrize("go,ge,local", MODES)
def test_score_related_pairs(engine, golden, n, go, ge, local):
    import oracle
    Y, X = related_pair(n, n + 17)
    r = engine.score(Y, X, golden.blosum62, go, ge, local)
    assert (r["score"], r["i_end"], r["j_end"]) == oracle.score_ag(Y, X, golden.blosum62, go, ge, local)


def test_empty_and_invalid(engine, golden):
    import oracle
    for R, C in [(0, 0), (0, 9), (7, 0)]:
        Y, X = random_pair(R, C, 1)
        for go, ge, local in MODES:
            r = engine.score(Y, X, golden.blosum62, go, ge, local)
            assert (r["score"], r["i_end"], r["j_end"]) == oracle.score_ag(Y, X, golden.blosum62, go, ge, local)
    Y, X = random_pair(10, 10, 2)
    for go, ge in [(-1, -11), (-3, 2)]:
        with pytest.raises(gsa.NwError):
            engine.score(Y, X, golden.blosum62, go, ge, False)


def test_linear_global_equals_strip_fill(engine, golden):
    """go == ge == g, global = the reference's NW-LG: same align_cost as the strip fill (config 2 pair)."""
    Y, X = golden.pair("len12124[:10000] len15390[:10000]")
    assert engine.score(Y, X, golden.blosum62, -11)["score"] == -4922
    for k in golden.known["cases"]:
        Y, X = golden.pair(k["pair"])
        assert engine.score(Y, X, golden.blosum62, -11)["score"] == k["align_cost"]


@pytest.mark.parametrize("go,ge,local", [(-11, -11, True), (-11, -1, False)])
def test_config5_50k(engine, golden, go, ge, local):
    """BASELINE configs[4]: 50k x 50k random pair (seed 200), SW-LG and NW-AG, against the
    oracle's tiled OpenMP restatement (bit-identical to its row-streaming one)."""
    import oracle
    from gpuseqalign_amd import formats as F
    Y, X = F.synthetic_seq(50000, 200), F.synthetic_seq(50000, 201)
    r = engine.score(Y, X, golden.blosum62, go, ge, local)
    ref = oracle.score_ag(Y, X, golden.blosum62, go, ge, local, mt=True, blocksz=256, nthreads=16)
    assert (r["score"], r["i_end"], r["j_end"]) == ref


@pytest.mark.parametrize("R,C", [(1, 300), (700, 130), (2049, 1500)])
@pytest.mark.parametrize("go,ge,local", MODES)
def test_row_scan_path(engine, golden, R, C, go, ge, local, monkeypatch, knobs):
    """Scores normally run on the strip kernel (affine / local modes); GSA_SCORE_SCAN=1 keeps the
    row-scan kernel reachable: both equal the oracle."""
    import oracle
    knobs("GSA_SCORE_SCAN", "1")
    Y, X = random_pair(R, C, 5 * R + C)
    r = engine.score(Y, X, golden.blosum62, go, ge, local)
    assert (r["score"], r["i_end"], r["j_end"]) == oracle.score_ag(Y, X, golden.blosum62, go, ge, local)


@pytest.mark.parametrize("go,ge", [(-11, -11), (-11, -1), (-5, -2)])
@pytest.mark.parametrize("gapR", [0, 37, 250, 3000])
def test_local_ties_first_in_row_major(engine, golden, go, ge, gapR):
    """SW: the same motif twice in Y (rows apart, across strip boundaries for the larger gaps),
    flanked by a letter that scores -4 against everything (match +5, mismatch -4): two equal
    maxima; the end cell reported is the first in row-major order, as the oracle's strict '>'
    row sweep keeps."""
    import oracle
    n = int(round(np.sqrt(golden.blosum62.size)))
    sub = np.full((n, n), -4, np.int32)
    np.fill_diagonal(sub[:20, :20], 5)
    sub = sub.reshape(golden.blosum62.shape)
    rng = np.random.default_rng(gapR + 7)
    motif = rng.integers(0, 20, 300).astype(np.int32)
    fl = lambda k: np.full(k, 22, np.int32)
    Y = np.concatenate([[0], fl(5), motif, fl(gapR + 1), motif, fl(9)]).astype(np.int32)
    X = np.concatenate([[0], fl(50), motif, fl(40)]).astype(np.int32)
    r = engine.score(Y, X, sub, go, ge, True)
    ref = oracle.score_ag(Y, X, sub, go, ge, True)
    assert ref == (1500, 305, 350)
    assert (r["score"], r["i_end"], r["j_end"]) == ref


def test_local_all_mismatch(engine, golden):
    """SW with no positive cell: (0, 0, 0)."""
    import oracle
    sub = np.full_like(golden.blosum62, -4)
    Y, X = random_pair(900, 1300, 3)
    r = engine.score(Y, X, sub, -11, -1, True)
    assert (r["score"], r["i_end"], r["j_end"]) == (0, 0, 0) == oracle.score_ag(Y, X, sub, -11, -1, True)


def test_local_fallbacks_to_row_scan(engine, golden):
    """SW takes the row scan when the strip kernel's conditions fail: go == 0 (cells past C could
    tie the maximum) and scores >= 2^26 (the kernel flags them; packed with the step they would
    wrap).  Both equal the oracle."""
    import oracle
    Y, X = random_pair(700, 900, 11)
    for go, ge in [(0, 0)]:
        r = engine.score(Y, X, golden.blosum62, go, ge, True)
        assert (r["score"], r["i_end"], r["j_end"]) == oracle.score_ag(Y, X, golden.blosum62, go, ge, True)
    n = int(round(np.sqrt(golden.blosum62.size)))
    sub = np.full((n, n), -30000, np.int32)
    np.fill_diagonal(sub, 30000)
    sub = sub.reshape(golden.blosum62.shape)
    Y, _ = random_pair(2600, 10, 12)
    X = Y.copy()
    ref = oracle.score_ag(Y, X, sub, -11, -1, True)
    assert ref[0] >= 1 << 26
    r = engine.score(Y, X, sub, -11, -1, True)
    assert (r["score"], r["i_end"], r["j_end"]) == ref


@pytest.mark.parametrize("R,C", [(300, 1), (65, 63), (700, 130), (1500, 1000)])
@pytest.mark.parametrize("go,ge,local", MODES)
def test_strip_kernel_path(engine, golden, R, C, go, ge, local, monkeypatch, knobs):
    """GSA_SCORE_KERNEL=strip: the strip kernel's score modes (nw_strip.hip), kept reachable beside
    the K-rows score kernel (nw_kscore.hip) that runs by default."""
    import oracle
    knobs("GSA_SCORE_KERNEL", "strip")
    Y, X = random_pair(R, C, 7 * R + C)
    r = engine.score(Y, X, golden.blosum62, go, ge, local)
    assert (r["score"], r["i_end"], r["j_end"]) == oracle.score_ag(Y, X, golden.blosum62, go, ge, local)


@pytest.mark.parametrize("k", ["2", "4"])
@pytest.mark.parametrize("R", [2048, 2049, 2050, 2051, 2052, 3071])
@pytest.mark.parametrize("go,ge,local", MODES)
def test_result_row_positions(engine, golden, monkeypatch, k, R, go, ge, local, knobs):
    """The K-rows score kernel reads the NW result cell (R, C) from the lane and row that hold it
    (row kR = (R - r0) mod K of lane (R - r0) / K of a later ticket's strip): every kR, a strip's
    first and last rows, at K = 2 and 4 rows per lane (GSA_SCORE_K)."""
    import oracle
    knobs("GSA_SCORE_K", k)
    Y, X = random_pair(R, 257, R + 11)
    r = engine.score(Y, X, golden.blosum62, go, ge, local)
    assert (r["score"], r["i_end"], r["j_end"]) == oracle.score_ag(Y, X, golden.blosum62, go, ge, local)


@pytest.mark.parametrize("substsz", [4, 25, 26, 32])
@pytest.mark.parametrize("go,ge,local", MODES)
def test_alphabet_sizes(engine, golden, substsz, go, ge, local):
    """Other alphabets: the K-rows score kernel's LDS holds a profile row per letter (substsz <= 25
    or so fits; 32 letters exceed the 160 KB and take the strip kernel), so every path is reached."""
    import oracle
    rng = np.random.default_rng(substsz * 100 + 7)
    sub = rng.integers(-6, 12, size=(substsz, substsz)).astype(np.int32)
    Y, X = random_pair(1500, 1100, substsz + 5, alphabet=substsz)
    r = engine.score(Y, X, sub, go, ge, local)
    assert (r["score"], r["i_end"], r["j_end"]) == oracle.score_ag(Y, X, sub, go, ge, local)


@pytest.mark.parametrize("k", ["2", "4"])
@pytest.mark.parametrize("q8", ["0", "1", "2"])
@pytest.mark.parametrize("go,ge,local", MODES + [(-120, -120, False), (-120, -120, True), (-70, -60, False)])
def test_profile_widths_and_stale_columns(engine, golden, monkeypatch, q8, k, go, ge, local, knobs):
    """The K-rows score kernel's int16 and int8 column profiles (GSA_KROW_Q8 = 0 / 2; 1 = int8 for
    linear modes only), the int8 instance's decline for s - go - ge outside int8 (gap -120, -70/-60:
    the int16 instance runs), and columns right of C: a long pair first leaves real letters in the
    profile ring, then a short one's strips read the columns past C up to 16 NB - 1, which the
    profiler must have rebuilt with the NEG letter (SW tracks those cells; a stale profile there
    once gave SW-AG 64 x 65 the score 197).  Both strip heights: 2 and 4 rows per lane (GSA_SCORE_K;
    by default 4 for NW-LG, 2 otherwise), so the result cell falls at every row of a lane."""
    import oracle
    knobs("GSA_KROW_Q8", q8)
    knobs("GSA_SCORE_K", k)
    for R, C in [(3, 3000), (64, 65), (200, 3000), (65, 100), (1, 200), (64, 65)]:
        Y, X = random_pair(R, C, 11 * R + C)
        r = engine.score(Y, X, golden.blosum62, go, ge, local)
        assert (r["score"], r["i_end"], r["j_end"]) == oracle.score_ag(Y, X, golden.blosum62, go, ge, local), (R, C)


@pytest.mark.parametrize("k", ["2", "4"])
@pytest.mark.parametrize("q8", ["0", "1"])
@pytest.mark.parametrize("go,ge,local", MODES)
def test_score_both_ends(engine, golden, monkeypatch, k, q8, go, ge, local, knobs):
    """NW from both ends (gsa_capi.hip score_bidi, nw_bidi.hip), forced at every size
    (GSA_SCORE_BIDI=2; by default pairs whose halves keep >= 4 tickets): the top half's tap row m,
    the reversed bottom half's row R - m and the combine.  Local modes with R % K == 0 take the
    three-pair SW from both ends (GSA_SCORE_BIDI_SW defaults to on); R % K != 0 keeps the
    one-direction kernel in every mode.  All equal the oracle."""
    import oracle
    knobs("GSA_SCORE_BIDI", "2")
    knobs("GSA_SCORE_K", k)
    knobs("GSA_KROW_Q8", q8)
    for R, C in [(2, 1), (4, 5), (8, 300), (130, 1), (130, 700), (512, 64), (514, 1000), (1024, 1024), (1027, 900),
                 (2052, 257), (4100, 3000)]:
        Y, X = random_pair(R, C, 13 * R + C)
        r = engine.score(Y, X, golden.blosum62, go, ge, local)
        assert (r["score"], r["i_end"], r["j_end"]) == oracle.score_ag(Y, X, golden.blosum62, go, ge, local), (R, C)


@pytest.mark.parametrize("k", ["2", "4"])
@pytest.mark.parametrize("go,ge", [(-11, -11), (-11, -1), (-5, -2), (-3, -1)])
@pytest.mark.parametrize("ins", [1, 7, 40, 300])
def test_score_both_ends_gap_across_split(engine, golden, monkeypatch, k, go, ge, ins, knobs):
    """A vertical gap that crosses the split row m = K floor(R / 2K): Y is X with ins letters
    inserted around the middle, so the best path's gap spans rows m and m + 1 and pays its open once
    (the combine's F + F^r - (go - ge) term); also a horizontal gap at the split (X longer)."""
    import oracle
    knobs("GSA_SCORE_BIDI", "2")
    knobs("GSA_SCORE_K", k)
    rng = np.random.default_rng(ins * 31 + int(k))
    base = rng.integers(0, 20, 1200).astype(np.int32)
    extra = rng.integers(0, 20, ins).astype(np.int32)
    for cut in (600 - ins // 2, 600 - ins + 2, 600):
        ycore = np.concatenate([base[:cut], extra, base[cut:]])
        Y = np.concatenate([[0], ycore]).astype(np.int32)
        X = np.concatenate([[0], base]).astype(np.int32)
        for A, B in ((Y, X), (X, Y)):
            A = A[:len(A) - (len(A) - 1) % int(k)]
            r = engine.score(A, B, golden.blosum62, go, ge, False)
            assert (r["score"], r["i_end"], r["j_end"]) == oracle.score_ag(A, B, golden.blosum62, go, ge, False), cut


def test_score_both_ends_default_matches_one_direction(engine, golden, monkeypatch, knobs):
    """The default switch (GSA_SCORE_BIDI=1: halves of >= 4 tickets) on a 20k related pair, NW-LG
    and NW-AG, against the one-direction kernel (GSA_SCORE_BIDI=0) and the oracle's tiled restatement."""
    import oracle
    Y, X = related_pair(20000, 20100)
    Y = Y[:len(Y) - (len(Y) - 1) % 4]  # R % K == 0: the split's rows are lanes' last rows
    for go, ge in [(-11, -11), (-11, -1)]:
        knobs("GSA_SCORE_BIDI", "1")
        r1 = engine.score(Y, X, golden.blosum62, go, ge, False)
        knobs("GSA_SCORE_BIDI", "0")
        r0 = engine.score(Y, X, golden.blosum62, go, ge, False)
        ref = oracle.score_ag(Y, X, golden.blosum62, go, ge, False, mt=True, blocksz=256, nthreads=8)
        assert (r1["score"], r1["i_end"], r1["j_end"]) == (r0["score"], r0["i_end"], r0["j_end"]) == ref


@pytest.mark.parametrize("k", ["2", "4"])
@pytest.mark.parametrize("go,ge", [(-11, -11), (-11, -1), (-4, -3)])
def test_score_both_ends_transposed(engine, golden, monkeypatch, k, go, ge, knobs):
    """R not a multiple of K but C one: the pair runs transposed from both ends (X down the rows, the
    table transposed), on an asymmetric table so a missed transpose shows; R and C both off the
    multiple keep one direction.  All equal the oracle, end cell (R, C)."""
    import oracle
    knobs("GSA_SCORE_BIDI", "2")
    knobs("GSA_SCORE_K", k)
    n = int(round(np.sqrt(golden.blosum62.size)))
    rng = np.random.default_rng(int(k) * 7 + go)
    sub = rng.integers(-7, 9, size=(n, n)).astype(np.int32)
    assert not np.array_equal(sub, sub.T)
    kk = int(k)
    for R, C in [(kk * 300 + 1, kk * 400), (kk * 513 + 1, kk * 41), (kk * 77 + 1, kk * 900 + 1), (kk * 2 + 1, kk * 2),
                 (kk * 4, 0), (0, kk * 4), (kk * 4, 1), (1, kk * 4), (kk * 2, kk * 2)]:
        Y, X = random_pair(R, C, 17 * R + C)
        r = engine.score(Y, X, sub, go, ge, False)
        assert (r["score"], r["i_end"], r["j_end"]) == oracle.score_ag(Y, X, sub, go, ge, False), (R, C)


def test_score_both_ends_random_shapes(engine, golden, monkeypatch, knobs):
    """40 random NW shapes (R, C in 1..3000, either parity), random gap pairs and tables, forced from
    both ends where the shape allows (GSA_SCORE_BIDI=2): equal to the oracle."""
    import oracle
    knobs("GSA_SCORE_BIDI", "2")
    n = int(round(np.sqrt(golden.blosum62.size)))
    rng = np.random.default_rng(2024)
    for case in range(40):
        R, C = (int(v) for v in rng.integers(1, 3001, 2))
        ge = -int(rng.integers(1, 6))
        go = ge - int(rng.integers(0, 12))
        sub = rng.integers(-8, 12, size=(n, n)).astype(np.int32)
        Y, X = random_pair(R, C, 1000 + case)
        r = engine.score(Y, X, sub, go, ge, False)
        assert (r["score"], r["i_end"], r["j_end"]) == oracle.score_ag(Y, X, sub, go, ge, False), (case, R, C, go, ge)


@pytest.mark.timeout(300)
def test_score_both_ends_100k(engine, golden, knobs):
    """100k x 100k NW-AG and NW-LG (default switch: from both ends) against the oracle's tiled OpenMP
    restatement (score_oracle.c, ~1e10 cells: seconds on the box's 16 threads) and against the
    one-direction kernel (GSA_SCORE_BIDI=0)."""
    import oracle
    from gpuseqalign_amd import formats as F
    Y, X = F.synthetic_seq(100000, 300), F.synthetic_seq(100000, 301)
    for go, ge in [(-11, -1), (-11, -11)]:
        knobs("GSA_SCORE_BIDI", "1")
        r1 = engine.score(Y, X, golden.blosum62, go, ge, False)
        knobs("GSA_SCORE_BIDI", "0")
        r0 = engine.score(Y, X, golden.blosum62, go, ge, False)
        ref = oracle.score_ag(Y, X, golden.blosum62, go, ge, False, mt=True)
        assert (r1["score"], r1["i_end"], r1["j_end"]) == ref, (go, ge)
        assert (r0["score"], r0["i_end"], r0["j_end"]) == ref, (go, ge)


@pytest.mark.parametrize("gran", ["0", "1"])
@pytest.mark.parametrize("skew", ["-1", "0", "700"])
def test_score_both_ends_granule_tap(engine, golden, monkeypatch, gran, skew, knobs):
    """The halves' meeting rows read from the last ticket's granules when a half ends on a ticket
    boundary (GSA_BIDI_GRAN=1, the default past 4 tickets: the top half always, the bottom when R
    is a multiple of the ticket too), or from lane taps on both sides (GSA_BIDI_GRAN=0); the top
    half's extra rows (GSA_BIDI_SKEW; -1 = the cost model) move the split.  Both NW modes, both
    rows-per-lane settings, R a multiple of the ticket (both halves free) and not; the oracle."""
    import oracle
    knobs("GSA_SCORE_BIDI", "2")
    knobs("GSA_BIDI_GRAN", gran)
    knobs("GSA_BIDI_SKEW", skew)
    for k in ("2", "4"):
        knobs("GSA_SCORE_K", k)
        for R, C in [(4096, 1500), (5120, 900), (4100, 2600), (6002, 700), (8192, 333)]:
            Y, X = random_pair(R, C, 29 * R + C)
            for go, ge in [(-11, -1), (-11, -11), (-4, -2)]:
                r = engine.score(Y, X, golden.blosum62, go, ge, False)
                assert (r["score"], r["i_end"], r["j_end"]) == oracle.score_ag(Y, X, golden.blosum62, go, ge, False), \
                    (k, R, C, go, ge)


def test_score_both_ends_large_random_shapes(engine, golden, monkeypatch, knobs):
    """Ten random shapes of 4k-30k rows and columns (both parities, both split forms: granule tap or
    lane taps, transposed when only C suits), random affine / linear gaps: the default path and the
    one-direction kernel (GSA_SCORE_BIDI=0) against the oracle's tiled OpenMP restatement."""
    import oracle
    rng = np.random.default_rng(77)
    for case in range(10):
        R, C = (int(v) for v in rng.integers(4000, 30001, 2))
        ge = -int(rng.integers(1, 4))
        go = ge - int(rng.integers(0, 12))
        Y, X = random_pair(R, C, 5000 + case)
        knobs("GSA_SCORE_BIDI", "1")
        r1 = engine.score(Y, X, golden.blosum62, go, ge, False)
        knobs("GSA_SCORE_BIDI", "0")
        r0 = engine.score(Y, X, golden.blosum62, go, ge, False)
        ref = oracle.score_ag(Y, X, golden.blosum62, go, ge, False, mt=True)
        assert (r1["score"], r1["i_end"], r1["j_end"]) == ref, (case, R, C, go, ge)
        assert (r0["score"], r0["i_end"], r0["j_end"]) == ref, (case, R, C, go, ge)


def _planted(R, C, seed, plants):
    """A random pair with identical segments planted: plants = [(row, col, length)] (1-based first
    row / column of the segment in Y / X), so the best local alignments sit where the test wants."""
    rng = np.random.default_rng(seed)  # (independent streams: random_pair's Y and X overlap when shifted)
    Y = np.concatenate([[0], rng.integers(0, 20, R)]).astype(np.int32)
    X = np.concatenate([[0], rng.integers(0, 20, C)]).astype(np.int32)
    for (r, c, n) in plants:
        seg = np.random.default_rng(1000 + n).integers(0, 20, n).astype(np.int32)  # equal n: equal segments
        Y[r:r + n] = seg
        X[c:c + n] = seg
    return Y, X


@pytest.mark.parametrize("k", ["2", "4"])
@pytest.mark.parametrize("go,ge", [(-11, -11), (-11, -1), (-5, -2)])
def test_score_local_both_ends(engine, golden, monkeypatch, capfd, k, go, ge, knobs):
    """SW from both ends (score_bidi, local: top forward, bottom reversed, bottom forward from a
    fresh border): best alignments planted wholly in the top half, wholly in the bottom, across the
    split row m (back to one direction), tied in both halves and twice in the bottom (first in
    row-major), and plain random pairs; every result equals the oracle, and the log names the way
    each pair went."""
    import oracle
    knobs("GSA_SCORE_BIDI", "2")
    knobs("GSA_SCORE_K", k)
    knobs("GSA_BIDI_LOG", "1")
    kk = int(k)
    R, C = 1600 * kk // 2, 1300
    m = kk * (R // (2 * kk))
    cases = [([(100, 200, 60)], "answer"),                       # top half
             ([(m + 300, 700, 60)], "answer"),                   # bottom half
             ([(m - 30, 500, 60)], "one direction"),             # across row m
             # equal segments (tied scores; they also pair across, so either way may be taken)
             ([(200, 900, 50), (m + 200, 300, 50)], None),
             ([(m + 100, 1000, 50), (m + 400, 100, 50)], None)]
    for i, (plants, way) in enumerate(cases):
        Y, X = _planted(R, C, 40 + i, plants)
        capfd.readouterr()
        r = engine.score(Y, X, golden.blosum62, go, ge, True)
        assert (r["score"], r["i_end"], r["j_end"]) == oracle.score_ag(Y, X, golden.blosum62, go, ge, True), (i, plants)
        err = capfd.readouterr().err
        # (at -5/-2 random letters align in the linear regime: long alignments that cross m)
        assert "gsa local both ends" in err and (way is None or go == -5 or f"-> {way}" in err), (i, plants, err)
    for R2, C2 in [(2, 1), (4, 5), (130, 700), (1024, 1024), (2052, 257), (4100, 3000)]:
        R2 -= R2 % kk
        Y, X = random_pair(R2, C2, 11 * R2 + C2)
        r = engine.score(Y, X, golden.blosum62, go, ge, True)
        assert (r["score"], r["i_end"], r["j_end"]) == oracle.score_ag(Y, X, golden.blosum62, go, ge, True), (R2, C2)


def test_score_local_both_ends_default_matches_one_direction(engine, golden, monkeypatch, knobs):
    """The default switch on SW (halves of >= 4 tickets, R even): random 6k-20k shapes and a related
    20k pair (its alignment crosses the split: one direction), against GSA_SCORE_BIDI_SW=0."""
    rng = np.random.default_rng(91)
    pairs = [random_pair(int(a) * 2, int(b), 700 + i) for i, (a, b) in enumerate(rng.integers(3000, 10001, (6, 2)))]
    Yr, Xr = related_pair(20000, 20100)
    pairs.append((Yr[:len(Yr) - (len(Yr) - 1) % 2], Xr))
    for Y, X in pairs:
        for go, ge in [(-11, -11), (-11, -1)]:
            knobs("GSA_SCORE_BIDI_SW", None)
            r1 = engine.score(Y, X, golden.blosum62, go, ge, True)
            knobs("GSA_SCORE_BIDI_SW", "0")
            r0 = engine.score(Y, X, golden.blosum62, go, ge, True)
            assert (r1["score"], r1["i_end"], r1["j_end"]) == (r0["score"], r0["i_end"], r0["j_end"]), (len(Y), len(X))


@pytest.mark.parametrize("k", ["2", "4"])
@pytest.mark.parametrize("go,ge", [(-11, -11), (-11, -1)])
def test_score_local_both_ends_continuation(engine, golden, monkeypatch, capfd, k, go, ge, knobs):
    """SW from both ends whose best alignment crosses the split, on a pair long enough for the top half
    to end on a ticket boundary: the way back continues the pair from that ticket in a second launch
    (its row above the top's last-ticket granules, restamped) instead of the whole one-direction run;
    crossing alignments planted at three places around the split row and one in the bottom only,
    equal to the oracle, and the log shows the way taken (GSA_BIDI_SW_CONT=0: the whole run again,
    same result)."""
    import oracle
    knobs("GSA_SCORE_K", k)
    knobs("GSA_BIDI_LOG", "1")
    kk = int(k)
    R, C = 3000 * kk, 1500
    for i, (dr, way) in enumerate([(-40, "bottom again"), (-5, "bottom again"), (-75, "bottom again"),
                                   (900, "answer")]):
        capfd.readouterr()
        engine.set_knob("GSA_BIDI_SW_CONT", None)
        Y, X = _planted(R, C, 60 + i, [(0, 0, 0)])
        r = engine.score(Y, X, golden.blosum62, go, ge, True)
        assert (r["score"], r["i_end"], r["j_end"]) == oracle.score_ag(Y, X, golden.blosum62, go, ge, True), i
        m = int(capfd.readouterr().err.split(" m ")[1].split(",")[0])
        Y, X = _planted(R, C, 60 + i, [(m + dr, 400 + 100 * i, 80)])
        ref = oracle.score_ag(Y, X, golden.blosum62, go, ge, True)
        r = engine.score(Y, X, golden.blosum62, go, ge, True)
        err = capfd.readouterr().err
        assert (r["score"], r["i_end"], r["j_end"]) == ref, (i, m, err)
        assert f"-> {way}" in err, (i, m, err)
        knobs("GSA_BIDI_SW_CONT", "0")
        r0 = engine.score(Y, X, golden.blosum62, go, ge, True)
        assert (r0["score"], r0["i_end"], r0["j_end"]) == ref, (i, m)
        assert ("-> one direction" if way != "answer" else "-> answer") in capfd.readouterr().err, (i, m)
