#!/usr/bin/env python3
"""Generate the size-scale golden fixtures from the oracle (CPU, this container).

  tests/golden/config3_100k.json -- BASELINE configs[2]: the 100k x 100k related pair
      (seqX = splitmix64 seed 100, seqY = seqX mutated with seed 101) and the
      unrelated pair seed 102/103.  align_cost, score hash (NwHash2_Sparse == NwHash1_Plain,
      nwtrace2_sparse.cpp:263-340), Trace2 hash + edit-string digest (nwtrace2_sparse.cpp:
      102-257) and a digest of every tile-header word for the geometries the engine uses.
      The oracle works in O(headers) memory: orc_sparse_headers streams two rows.
  tests/golden/config4_pairs.json -- BASELINE configs[3]: 512 pairs, lengths uniform in
      [18000, 22000] (shard.synthetic_batch, seeds 1000+k); align_cost and score hash of
      each pair from the streaming cpu1 restatement (orc_hash_stream).

      Plus sha256 digests of the tile headers of 16 of the pairs (tileBx 256).
  tests/golden/config5_50k.json -- BASELINE configs[4]: the 50k x 50k random pair (seeds 200/201),
      score-only SW/NW x linear/affine gaps (oracle/score_oracle.c), score and end cell.

Test infrastructure: the oracle is the checker.
Run:  python tools/make_goldens.py [config3|config4|config4_headers|config5]
"""
import hashlib
import json
import os
import sys
import time
from multiprocessing import Pool

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np

GOLDEN = os.path.join(ROOT, "tests", "golden")


def _subst():
    from gpuseqalign_amd import formats as F
    return F.read_subst_json(os.path.join(GOLDEN, "resrc", "subst.json")).matrix("blosum62")


def config3_pairs():
    from gpuseqalign_amd import formats as F
    X = F.synthetic_seq(100000, 100)
    Y = F.mutate_seq(X, 101)
    return {"related": (Y, X), "unrelated": (F.synthetic_seq(100000, 102), F.synthetic_seq(100000, 103))}


def header_digest(hrow, hcol):
    h = hashlib.sha256()
    h.update(np.ascontiguousarray(hrow, np.int32).tobytes())
    h.update(np.ascontiguousarray(hcol, np.int32).tobytes())
    return h.hexdigest()


def make_config3(geoms=((1024, 256),)):
    import oracle
    sub = _subst()
    out = {"_about": "oracle goldens for BASELINE configs[2] (tools/make_goldens.py); blosum62, gapo -11",
           "pairs": {}}
    for name, (Y, X) in config3_pairs().items():
        t0 = time.time()
        sh, cost = oracle.hash_stream(Y, X, sub, -11)
        rec = {"R": len(Y) - 1, "C": len(X) - 1, "align_cost": cost, "score_hash": "%08x" % sh,
               "seqY_sha256": hashlib.sha256(Y.tobytes()).hexdigest(),
               "seqX_sha256": hashlib.sha256(X.tobytes()).hexdigest(), "headers": {}}
        for tBy, tBx in geoms:
            hr, hc, tr, tc, c2 = oracle.sparse_headers(Y, X, sub, -11, tBy, tBx)
            assert c2 == cost
            th, edit, c3 = oracle.trace_sparse(hr, hc, tr, tc, tBy, tBx, Y, X, sub, -11)
            assert c3 == cost
            rec["trace_hash"] = "%08x" % th
            rec["edit_trace_len"] = len(edit)
            rec["edit_trace_sha256"] = hashlib.sha256(edit.encode()).hexdigest()
            rec["edit_trace_head"] = edit[:64]
            rec["headers"]["%dx%d" % (tBy, tBx)] = {"trows": tr, "tcols": tc, "sha256": header_digest(hr, hc)}
            del hr, hc
        print(name, rec["align_cost"], rec["trace_hash"], "%.1fs" % (time.time() - t0), flush=True)
        out["pairs"][name] = rec
    with open(os.path.join(GOLDEN, "config3_100k.json"), "w") as f:
        json.dump(out, f, indent=1)


def _cfg4_one(k):
    import oracle
    from gpuseqalign_amd import shard
    Y, X = shard.synthetic_batch(1, 18000, 22000, seed0=1000 + k)[0]
    sh, cost = oracle.hash_stream(Y, X, _subst(), -11)
    return k, len(Y) - 1, len(X) - 1, cost, sh


CFG4_HDR_PAIRS = list(range(0, 512, 32))  # 16 pairs spread over the batch
CFG4_HDR_TBX = 256


def _cfg4_hdr(k):
    import oracle
    from gpuseqalign_amd import shard
    Y, X = shard.synthetic_batch(1, 18000, 22000, seed0=1000 + k)[0]
    hr, hc, tr, tc, cost = oracle.sparse_headers(Y, X, _subst(), -11, 1024, CFG4_HDR_TBX)
    return k, cost, header_digest(hr, hc)


def make_config4_headers(procs=8):
    """Tile-header digests of 16 config-4 pairs (tileBy 1024, tileBx 256) added to
    config4_pairs.json: the batch's header words at full size, on whatever strip geometry
    the batch runs."""
    path = os.path.join(GOLDEN, "config4_pairs.json")
    with open(path) as f:
        out = json.load(f)
    t0 = time.time()
    with Pool(procs) as p:
        res = sorted(p.map(_cfg4_hdr, CFG4_HDR_PAIRS))
    for k, cost, _ in res:
        assert cost == out["align_cost"][k]
    out["headers"] = {"tileBy": 1024, "tileBx": CFG4_HDR_TBX, "pairs": [r[0] for r in res],
                      "sha256": [r[2] for r in res]}
    with open(path, "w") as f:
        json.dump(out, f)
    print("config4 headers: %d pairs, %.1fs" % (len(res), time.time() - t0))


CFG5_MODES = [("SW-LG", -11, -11, True), ("NW-AG", -11, -1, False), ("SW-AG", -11, -1, True), ("NW-LG", -11, -11, False)]


def make_config5(procs=8):
    """BASELINE configs[4]: the 50k x 50k random pair (seeds 200/201), score-only, from the
    oracle's tiled OpenMP restatement of score_oracle.c (bit-identical to its streaming one)."""
    import oracle
    from gpuseqalign_amd import formats as F
    Y, X = F.synthetic_seq(50000, 200), F.synthetic_seq(50000, 201)
    sub = _subst()
    out = {"_about": "oracle goldens for BASELINE configs[4] (tools/make_goldens.py): score_oracle.c, blosum62; "
                     "seqY = synthetic_seq(50000, 200), seqX = synthetic_seq(50000, 201)",
           "R": len(Y) - 1, "C": len(X) - 1, "seqY_sha256": hashlib.sha256(Y.tobytes()).hexdigest(),
           "seqX_sha256": hashlib.sha256(X.tobytes()).hexdigest(), "modes": {}}
    for name, go, ge, local in CFG5_MODES:
        t0 = time.time()
        sc, i, j = oracle.score_ag(Y, X, sub, go, ge, local, mt=True, blocksz=256, nthreads=procs)
        out["modes"][name] = {"gapo": go, "gape": ge, "local": local, "score": sc, "i_end": i, "j_end": j}
        print(name, sc, i, j, "%.1fs" % (time.time() - t0), flush=True)
    with open(os.path.join(GOLDEN, "config5_50k.json"), "w") as f:
        json.dump(out, f, indent=1)


def make_config4(n=512, procs=8):
    t0 = time.time()
    with Pool(procs) as p:
        res = sorted(p.map(_cfg4_one, range(n), chunksize=4))
    out = {"_about": "oracle goldens for BASELINE configs[3] (tools/make_goldens.py): shard.synthetic_batch("
                     "%d, 18000, 22000, seed0=1000); blosum62, gapo -11; cpu1 streaming restatement" % n,
           "n_pairs": n, "R": [r[1] for r in res], "C": [r[2] for r in res],
           "align_cost": [r[3] for r in res], "score_hash": ["%08x" % r[4] for r in res]}
    with open(os.path.join(GOLDEN, "config4_pairs.json"), "w") as f:
        json.dump(out, f)
    print("config4: %d pairs, %.1fs" % (n, time.time() - t0))


if __name__ == "__main__":
    what = sys.argv[1:] or ["config3", "config4"]
    if "config3" in what:
        make_config3()
    if "config4" in what:
        make_config4()
    if "config4" in what or "config4_headers" in what:
        make_config4_headers()
    if "config5" in what:
        make_config5()
