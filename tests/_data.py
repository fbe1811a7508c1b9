"""Golden inputs shared by the tests (reference data files copied under tests/golden/resrc)."""
import json
import os

import numpy as np

from gpuseqalign_amd import formats as F

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
RESRC = os.path.join(GOLDEN, "resrc")


class Golden:
    def __init__(self):
        self.subst_data = F.read_subst_json(os.path.join(RESRC, "subst.json"))
        self.seqs = F.read_fasta(os.path.join(RESRC, "seq_generated.fa"), self.subst_data.letter_map)
        with open(os.path.join(GOLDEN, "known_answers.json")) as f:
            self.known = json.load(f)
        self.blosum62 = self.subst_data.matrix("blosum62")

    def pair(self, line):
        p = F.parse_pair_line(line, self.seqs)
        return F.pair_arrays(p, self.seqs)

    def pairs(self, fname):
        return [(p, *F.pair_arrays(p, self.seqs)) for p in F.read_seq_pairs(os.path.join(RESRC, fname), self.seqs)]


def random_pair(R, C, seed, alphabet=20):
    """Synthetic pair (splitmix64 letters)."""
    return F.synthetic_seq(R, seed, alphabet), F.synthetic_seq(C, seed + 1, alphabet)


def related_pair(n, seed):
    x = F.synthetic_seq(n, seed)
    return F.mutate_seq(x, seed + 1), x
