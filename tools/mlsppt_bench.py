"""mlsppt vs mlsp end to end (host buffers, BASELINE configs[2] 100k x 100k related pair, tileBx 256):
the sum of the align laps (alloc + cpy_dev + init_hdr + calc + cpy_host, the reference's TSV
columns) and the wall time of the call, alternating the two paths; every result's align_cost
checked against the golden.  One JSON line per call, then a summary line."""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import gpuseqalign_amd as gsa
import bench

Y, X = bench.config3_pair()
sub = bench.subst_blosum62()
gold = bench.load_golden("config3_100k.json")["pairs"]["related"]["align_cost"]
eng = gsa.Engine(0)
res = {False: [], True: []}
for it in range(int(sys.argv[1]) if len(sys.argv) > 1 else 5):
    for ov in (False, True):
        t = time.perf_counter()
        r = eng.align_sparse(Y, X, sub, -11, tileBx=256, overlap=ov)
        wall = 1e3 * (time.perf_counter() - t)
        laps = {k: round(v, 3) for k, v in r.laps.items()}
        tot = sum(v for k, v in r.laps.items() if k.startswith("align."))
        assert r.align_cost == gold, (r.align_cost, gold)
        if it > 0:
            res[ov].append((tot, wall))
        print(json.dumps({"path": "mlsppt" if ov else "mlsp", "laps_total_ms": round(tot, 3), "wall_ms": round(wall, 2),
                          "laps": laps, "align_cost": r.align_cost}), flush=True)
m = {ov: np.median([x[0] for x in v]) for ov, v in res.items()}
w = {ov: np.median([x[1] for x in v]) for ov, v in res.items()}
print(json.dumps({"summary": "median over calls 2..", "mlsp_laps_ms": round(m[False], 3), "mlsppt_laps_ms": round(m[True], 3),
                  "ratio_laps": round(m[True] / m[False], 3), "mlsp_wall_ms": round(w[False], 2),
                  "mlsppt_wall_ms": round(w[True], 2), "ratio_wall": round(w[True] / w[False], 3)}), flush=True)
