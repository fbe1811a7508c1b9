"""Timing of the device-side consumers at BASELINE configs[2] (100k x 100k related pair):
sparse fill, header check (gsa_check_sparse_dev), device traceback (gsa_trace_sparse_dev)
against the host traceback (gsa_trace_sparse after copying the headers back); and the 10k
full fill + cell check.  One JSON line per measurement."""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import gpuseqalign_amd as gsa
from gpuseqalign_amd import formats as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sd = F.read_subst_json(os.path.join(ROOT, "tests", "golden", "resrc", "subst.json"))
sub = sd.matrix("blosum62")
eng = gsa.Engine(0)
dev = torch.device("cuda:0")
d = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.int32)).to(dev)


def timed(fn, reps=3):
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t = time.perf_counter()
        r = fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t)
    return r, 1e3 * min(ts)


for n, tBx in [(100000, 256), (100000, 512), (50000, 1024)]:
    X = F.synthetic_seq(n, 100)
    Y = F.mutate_seq(X, 101)
    geom = gsa.sparse_geometry(len(Y), len(X), tBx)
    y, x, s = d(Y), d(X), d(sub)
    hr = torch.empty(geom.hrowElems, dtype=torch.int32, device=dev)
    hc = torch.empty(geom.hcolElems, dtype=torch.int32, device=dev)
    args = (y.data_ptr(), len(Y), x.data_ptr(), len(X), s.data_ptr(), 25, -11)
    _, t_fill = timed(lambda: (eng.fill_sparse_dev(*args, tBx, hr.data_ptr(), hc.data_ptr()), eng.sync()))
    chk, t_chk = timed(lambda: eng.check_sparse_dev(*args, geom, hr.data_ptr(), hc.data_ptr()))
    tr_dev, t_trd = timed(lambda: eng.trace_sparse_dev(*args, geom, hr.data_ptr(), hc.data_ptr()))

    def host_trace():
        res = gsa.SparseResult(hr.cpu().numpy(), hc.cpu().numpy(), geom, 0, {})
        return gsa.trace_sparse(res, Y, X, sub, -11)
    tr_host, t_trh = timed(host_trace, reps=1)
    assert tr_dev == tr_host and chk["mismatches"] == 0
    cells = (len(Y) - 1) * (len(X) - 1)
    print(json.dumps({"R": len(Y) - 1, "C": len(X) - 1, "tileBx": tBx, "fill_ms": round(t_fill, 3),
                      "fill_tcups": round(cells / t_fill / 1e9, 3), "check_ms": round(t_chk, 3),
                      "check_values": chk["checked"], "check_gcups_equiv": round(cells / t_chk / 1e6, 1),
                      "trace_dev_ms": round(t_trd, 3), "trace_host_ms_incl_d2h": round(t_trh, 3),
                      "edit_len": len(tr_dev[1]), "align_cost": tr_dev[2]}), flush=True)

Yg, Xg = F.synthetic_seq(10000, 2), F.synthetic_seq(10000, 3)
y, x, s = d(Yg), d(Xg), d(sub)
out = torch.empty(len(Yg) * len(Xg), dtype=torch.int32, device=dev)
args = (y.data_ptr(), len(Yg), x.data_ptr(), len(Xg), s.data_ptr(), 25, -11)
_, t_fill = timed(lambda: (eng.fill_full_dev(*args, out.data_ptr()), eng.sync()))
chk, t_chk = timed(lambda: eng.check_full_dev(*args, out.data_ptr()))
print(json.dumps({"R": 10000, "C": 10000, "full_fill_ms": round(t_fill, 3), "full_check_ms": round(t_chk, 3),
                  "check_GBps": round(2 * 4 * out.numel() / t_chk / 1e6, 1), **chk}), flush=True)

# mlsppt: end-to-end host-buffer sparse align, plain vs overlapped copy-back (BASELINE configs[2])
X = F.synthetic_seq(100000, 100)
Y = F.mutate_seq(X, 101)
for ov in (False, True, False, True):
    t = time.perf_counter()
    r = eng.align_sparse(Y, X, sub, -11, tileBx=256, overlap=ov)
    tot = time.perf_counter() - t
    print(json.dumps({"mlsp": "mlsppt" if ov else "mlsp", "R": 100000, "wall_ms": round(1e3 * tot, 2),
                      "laps": {k: round(v, 3) for k, v in r.laps.items()}, "align_cost": r.align_cost}), flush=True)
