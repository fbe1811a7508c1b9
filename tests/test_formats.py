"""Input formats (mirrors of src/file_formats.cpp and src/benchmark.cpp:14-36)."""
import os

import numpy as np
import pytest

from gpuseqalign_amd import formats as F
from tests._data import RESRC


def test_subst_json(golden):
    sd = golden.subst_data
    assert sd.substsz == 25 and list(sd.letter_map)[:3] == ["A", "R", "N"]
    assert set(sd.subst_map) == {"blosum45", "blosum50", "blosum62", "blosum80", "blosum90"}
    b62 = sd.matrix("blosum62").reshape(25, 25)
    assert b62[0, 0] == 4 and b62[4, 4] == 9 and (b62 == b62.T).all()


def test_fasta_header_element(golden):
    s = golden.seqs["len1"].seq
    assert s[0] == 0 and len(s) == 2 and s[1] == golden.subst_data.letter_map["M"]
    assert len(golden.seqs["len23728"].seq) == 23729
    assert len(golden.seqs) == 32


def test_pairs_and_ranges(golden):
    pairs = F.read_seq_pairs(os.path.join(RESRC, "pair_debug.txt"), golden.seqs)
    assert len(pairs) == 173
    ph = F.read_seq_pairs(os.path.join(RESRC, "pair_phases.txt"), golden.seqs)
    p = [q for q in ph if q.seqY_range.r_not_default][0]
    assert p.seqY_range.l == 0 and not p.seqY_range.l_not_default
    Y, X = F.pair_arrays(p, golden.seqs)
    assert len(Y) == p.seqY_range.r + 1 and Y[0] == 0
    assert np.array_equal(Y[1:], golden.seqs[p.seqY_id].seq[1:1 + p.seqY_range.r])
    assert p.seqY_range.to_string(p.seqY_id) == f"{p.seqY_id}[:{p.seqY_range.r}]"


def test_range_errors(golden):
    with pytest.raises(F.NwFormatError):
        F.parse_pair_line("len8[5:3] len8", golden.seqs)
    with pytest.raises(F.NwFormatError):
        F.parse_pair_line("len8[:9] len8", golden.seqs)
    with pytest.raises(F.NwFormatError):
        F.parse_pair_line("nosuch len8", golden.seqs)


def test_fasta_bad_letter(tmp_path, golden):
    p = tmp_path / "bad.fa"
    p.write_text(">a\nMQ1\n")
    with pytest.raises(F.NwFormatError):
        F.read_fasta(str(p), golden.subst_data.letter_map)


def test_synthetic_is_deterministic():
    a = F.synthetic_seq(1000, 100)
    b = F.synthetic_seq(1000, 100)
    assert np.array_equal(a, b) and a[0] == 0 and a[1:].min() >= 0 and a[1:].max() <= 19
    g = F.splitmix64(100)
    first = [next(g) % 20 for _ in range(5)]
    assert list(a[1:6]) == first
