"""Input formats of the reference driver, restated for the host side.

Mirrors markods/GpuSeqAlign's parsers:
  * substitution-matrix JSON with comments (src/io.hpp:16-49 readFromJsonFile,
    comments allowed at :33; validation src/cmd_parser.cpp:316-355),
  * FASTA with a dummy header element 0 prepended to every sequence
    (src/file_formats.cpp:143-239, header element at :43-47),
  * pair lists with optional ``id[l:r]`` substring ranges
    (src/file_formats.cpp:241-399),
  * substring extraction with header (src/benchmark.cpp:14-36
    vectorSubstringWithHeader).

Errors raise ``NwFormatError`` carrying the reference's ``path:line:col: message``
shape (src/file_formats.cpp:15-31).
"""
from __future__ import annotations

import dataclasses
import json
import re
from collections import OrderedDict
from typing import Dict, List, Optional, Tuple

import numpy as np


class NwFormatError(ValueError):
    pass


def _strip_json_comments(text: str) -> str:
    """Remove // and /* */ comments outside string literals (nlohmann ignore_comments)."""
    out = []
    i, n = 0, len(text)
    in_str = False
    while i < n:
        c = text[i]
        if in_str:
            out.append(c)
            if c == "\\" and i + 1 < n:
                out.append(text[i + 1])
                i += 2
                continue
            if c == '"':
                in_str = False
            i += 1
            continue
        if c == '"':
            in_str = True
            out.append(c)
            i += 1
        elif text.startswith("//", i):
            j = text.find("\n", i)
            i = n if j < 0 else j
        elif text.startswith("/*", i):
            j = text.find("*/", i + 2)
            if j < 0:
                raise NwFormatError("unterminated /* comment")
            i = j + 2
        else:
            out.append(c)
            i += 1
    return "".join(out)


@dataclasses.dataclass
class NwSubstData:
    letter_map: "OrderedDict[str, int]"
    subst_map: "OrderedDict[str, np.ndarray]"  # name -> int32 [substsz*substsz]

    def matrix(self, name: str) -> np.ndarray:
        if name not in self.subst_map:
            raise NwFormatError(f"unknown substitution matrix name: {name}")
        return self.subst_map[name]

    @property
    def substsz(self) -> int:
        return len(self.letter_map)


def read_subst_json(path: str) -> NwSubstData:
    """subst.json loader + the checks of src/cmd_parser.cpp:316-355."""
    with open(path, "r") as f:
        raw = json.loads(_strip_json_comments(f.read()), object_pairs_hook=OrderedDict)
    letter_map = OrderedDict((k, int(v)) for k, v in raw["letterMap"].items())
    n = len(letter_map)
    for idx, (letter, val) in enumerate(letter_map.items()):
        if len(letter) != 1:
            raise NwFormatError(f"{path}: letter '{letter}' must be a single character")
        if val != idx:
            raise NwFormatError(f"{path}: letter map values must be consecutive starting from 0")
    subst_map = OrderedDict()
    for name, vals in raw["substMap"].items():
        arr = np.asarray(vals, dtype=np.int32)
        if arr.size != n * n:
            raise NwFormatError(f"{path}: substitution matrix '{name}' must have {n}x{n} elements")
        subst_map[name] = arr
    return NwSubstData(letter_map, subst_map)


@dataclasses.dataclass
class NwSeq:
    id: str
    info: str
    seq: np.ndarray  # int32 letters, element 0 is the dummy header


def read_fasta(path: str, letter_map: Dict[str, int]) -> "OrderedDict[str, NwSeq]":
    """readFromFastaFormat (src/file_formats.cpp:143-239)."""
    seqs: "OrderedDict[str, NwSeq]" = OrderedDict()
    cur_id: Optional[str] = None
    cur_info = ""
    cur: List[int] = []
    state = "header"

    def flush():
        if cur_id is not None and cur:
            seqs[cur_id] = NwSeq(cur_id, cur_info, np.asarray(cur, dtype=np.int32))

    with open(path, "r") as f:
        for iline, line in enumerate(f):
            s = line.strip()
            if not s:
                continue
            if s.startswith(">"):
                if state == "sequence":
                    raise NwFormatError(f"{path}:{iline + 1}:1: expected sequence after header")
                flush()
                parts = s[1:].strip().split(None, 1)
                if not parts:
                    raise NwFormatError(f"{path}:{iline + 1}:2: expected sequence id after '>' symbol")
                cur_id = parts[0]
                if cur_id in seqs:
                    raise NwFormatError(f"{path}:{iline + 1}:2: duplicate sequence id")
                cur_info = parts[1].rstrip() if len(parts) > 1 else ""
                cur = [0]  # header element (src/file_formats.cpp:43-47)
                state = "sequence"
                continue
            if state == "header":
                raise NwFormatError(f"{path}:{iline + 1}:1: expected sequence header (>)")
            for icol, ch in enumerate(line.rstrip("\n")):
                if ch in letter_map:
                    cur.append(letter_map[ch])
                elif ch.isspace():
                    continue
                else:
                    raise NwFormatError(f"{path}:{iline + 1}:{icol + 1}: letter not found in substitution letters")
            state = "seq_or_header"
    if state == "sequence":
        raise NwFormatError(f"{path}: expected sequence after header")
    if state == "header":
        raise NwFormatError(f"{path}: expected sequence header (>)")
    flush()
    return seqs


@dataclasses.dataclass(frozen=True)
class NwRange:
    """src/run_types.hpp:26-35: l inclusive, r exclusive, with 'not default' flags."""
    l: int
    r: int
    l_not_default: bool = False
    r_not_default: bool = False

    def to_string(self, seq_id: str) -> str:
        """seqIdAndRangeToString (src/file_formats.cpp:432-453)."""
        if not (self.l_not_default or self.r_not_default):
            return seq_id
        return f"{seq_id}[{self.l if self.l_not_default else ''}:{self.r if self.r_not_default else ''}]"


@dataclasses.dataclass(frozen=True)
class NwSeqPair:
    seqY_id: str
    seqY_range: NwRange
    seqX_id: str
    seqX_range: NwRange


_ID_RANGE = re.compile(r"\s*([^\s\[]+)(?:\[\s*([+-]?\d+)?\s*:\s*([+-]?\d+)?\s*\])?")


def _parse_id_range(text: str, pos: int, seqs, path: str, iline: int) -> Tuple[str, NwRange, int]:
    m = _ID_RANGE.match(text, pos)
    if not m:
        raise NwFormatError(f"{path}:{iline + 1}:{pos + 1}: expected sequence id")
    sid = m.group(1)
    if sid not in seqs:
        raise NwFormatError(f"{path}:{iline + 1}:{pos + 1}: unknown sequence id")
    n = len(seqs[sid].seq) - 1
    l, r = 0, n
    lnd = rnd = False
    if m.group(2) is not None:
        l, lnd = int(m.group(2)), True
        if l < 0:
            raise NwFormatError(f"{path}:{iline + 1}: left bound must be non-negative")
        if l >= n:
            raise NwFormatError(f"{path}:{iline + 1}: left bound greater than or equal to sequence length")
    if m.group(3) is not None:
        r, rnd = int(m.group(3)), True
        if r <= l:
            raise NwFormatError(f"{path}:{iline + 1}: right bound must be greater than left")
        if r > n:
            raise NwFormatError(f"{path}:{iline + 1}: right bound greater than sequence length")
    return sid, NwRange(l, r, lnd, rnd), m.end()


def read_seq_pairs(path: str, seqs) -> List[NwSeqPair]:
    """readFromSeqPairFormat (src/file_formats.cpp:343-399)."""
    pairs = []
    with open(path, "r") as f:
        for iline, line in enumerate(f):
            text = line.rstrip("\n")
            if not text.strip():
                continue
            y, yr, pos = _parse_id_range(text, 0, seqs, path, iline)
            x, xr, pos = _parse_id_range(text, pos, seqs, path, iline)
            if text[pos:].strip():
                raise NwFormatError(f"{path}:{iline + 1}:{pos + 1}: expected next line")
            pairs.append(NwSeqPair(y, yr, x, xr))
    if not pairs:
        raise NwFormatError(f"{path}: expected at least one sequence pair")
    return pairs


def parse_pair_line(line: str, seqs) -> NwSeqPair:
    """One pair line (e.g. 'len12124[:10000] len15390[:10000]')."""
    y, yr, pos = _parse_id_range(line, 0, seqs, "<pair>", 0)
    x, xr, pos = _parse_id_range(line, pos, seqs, "<pair>", 0)
    return NwSeqPair(y, yr, x, xr)


def substring_with_header(seq: np.ndarray, rng: NwRange) -> np.ndarray:
    """vectorSubstringWithHeader (src/benchmark.cpp:14-36)."""
    n = len(seq) - 1
    if rng.l < 0 or rng.l >= n or rng.r <= rng.l or rng.r > n:
        raise NwFormatError("cannot take substring")
    if (not rng.l_not_default or rng.l == 0) and (not rng.r_not_default or rng.r == n):
        return seq
    out = np.empty(1 + rng.r - rng.l, dtype=np.int32)
    out[0] = 0
    out[1:] = seq[1 + rng.l:1 + rng.r]
    return out


def pair_arrays(pair: NwSeqPair, seqs) -> Tuple[np.ndarray, np.ndarray]:
    """(seqY, seqX) with header element, as the driver builds them (benchmark.cpp:410-426)."""
    return (substring_with_header(seqs[pair.seqY_id].seq, pair.seqY_range),
            substring_with_header(seqs[pair.seqX_id].seq, pair.seqX_range))


def splitmix64(seed: int):
    """The build's own PRNG for synthetic sequences."""
    state = seed & 0xFFFFFFFFFFFFFFFF
    mask = 0xFFFFFFFFFFFFFFFF
    while True:
        state = (state + 0x9E3779B97F4A7C15) & mask
        z = state
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & mask
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & mask
        yield z ^ (z >> 31)


def synthetic_seq(n: int, seed: int, alphabet: int = 20) -> np.ndarray:
    """Letters iid uniform over `alphabet` codes (0..19 = A..V in subst.json), with header.

    Vectorised splitmix64 (same stream as `splitmix64`)."""
    mask = np.uint64(0xFFFFFFFFFFFFFFFF)
    k = np.arange(1, n + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = (np.uint64(seed) + k * np.uint64(0x9E3779B97F4A7C15)) & mask
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    out = np.empty(n + 1, dtype=np.int32)
    out[0] = 0
    out[1:] = (z % np.uint64(alphabet)).astype(np.int32)
    return out


def mutate_seq(base: np.ndarray, seed: int, p_sub: float = 0.15, p_indel: float = 0.02,
               alphabet: int = 20) -> np.ndarray:
    """seqY = seqX mutated (15 % substitutions, 2 % indels), SURVEY.md 8d config 3."""
    rng = splitmix64(seed)
    out = [0]
    for v in base[1:]:
        r = next(rng) / 2.0 ** 64
        if r < p_indel / 2:  # deletion
            continue
        if r < p_indel:  # insertion before
            out.append(int(next(rng) % alphabet))
        elif r < p_indel + p_sub:
            v = int(next(rng) % alphabet)
        out.append(int(v))
    return np.asarray(out, dtype=np.int32)
