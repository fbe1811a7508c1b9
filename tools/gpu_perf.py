"""Kernel timing probe: device-resident inputs, hipEvent timing on the launch stream."""
import os, sys, time, json, argparse
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import gpuseqalign_amd as gsa
from gpuseqalign_amd import formats as F

def run(eng, R, C, mode, tileBx=256, reps=5, seed=5):
    dev = torch.device("cuda:0")
    Y = torch.from_numpy(F.synthetic_seq(R, seed)).to(dev)
    X = torch.from_numpy(F.synthetic_seq(C, seed + 1)).to(dev)
    sd = F.read_subst_json(os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "resrc", "subst.json"))
    S = torch.from_numpy(sd.matrix("blosum62")).to(dev)
    st = torch.cuda.current_stream()
    if mode == "full":
        out = torch.empty((R + 1) * (C + 1), dtype=torch.int32, device=dev)
        fn = lambda: eng.fill_full_dev(Y.data_ptr(), R + 1, X.data_ptr(), C + 1, S.data_ptr(), 25, -11, out.data_ptr(), st.cuda_stream)
    else:
        g = gsa.sparse_geometry(R + 1, C + 1, tileBx)
        hr = torch.empty(g.hrowElems, dtype=torch.int32, device=dev)
        hc = torch.empty(g.hcolElems, dtype=torch.int32, device=dev)
        fn = lambda: eng.fill_sparse_dev(Y.data_ptr(), R + 1, X.data_ptr(), C + 1, S.data_ptr(), 25, -11, tileBx, hr.data_ptr(), hc.data_ptr(), st.cuda_stream)
    fn(); eng.sync(st.cuda_stream)
    ts = []
    for _ in range(reps):
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        e0.record(st); fn(); e1.record(st); eng.sync(st.cuda_stream)
        ts.append(e0.elapsed_time(e1))
    ms = float(np.median(ts))
    return {"R": R, "C": C, "mode": mode, "tileBx": tileBx, "ms": ms, "gcups": R * C / ms / 1e6, "all_ms": ts}

if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="2000,10000,23728")
    ap.add_argument("--shapes", default="252x4000,252x20000,504x20000,1008x20000")
    ap.add_argument("--big", type=int, default=0)
    a = ap.parse_args()
    eng = gsa.Engine(0)
    for sh in [x for x in a.shapes.split(",") if x]:
        R, C = map(int, sh.split("x"))
        for mode in ("full", "sparse"):
            print(json.dumps(run(eng, R, C, mode)), flush=True)
    for n in [int(x) for x in a.sizes.split(",")]:
        for mode in ("full", "sparse"):
            print(json.dumps(run(eng, n, n, mode)), flush=True)
    if a.big:
        print(json.dumps(run(eng, a.big, a.big, "sparse", tileBx=512, reps=3)), flush=True)
