#!/bin/bash
# A/B of library builds on the config-2 10k full fill and the 64-pair full batch: LIBS="head b"
# (gpuseqalign_amd/libgsa_<name>.so; cur = libgsa.so), each twice, interleaved.
cd ${GRAFT_REPO_ROOT:-/root/repo}
for rep in 1 2; do
  for lib in ${LIBS:-cur}; do
    L=$PWD/gpuseqalign_amd/libgsa.so; [ $lib != cur ] && L=$PWD/gpuseqalign_amd/libgsa_$lib.so
    GSA_LIB=$L timeout -k 10 120 python - <<'PY' || exit 1
import os, time, json, numpy as np, torch
import gpuseqalign_amd as gsa, bench
dev = torch.device("cuda:0")
eng = gsa.Engine(0)
Y, X = bench.config2_pair() if hasattr(bench, "config2_pair") else (None, None)
from gpuseqalign_amd import formats as F
if Y is None:
    Y, X = F.synthetic_seq(10000, 11), F.synthetic_seq(10000, 12)
sub = bench.subst_blosum62()
y, x, s = (torch.from_numpy(np.ascontiguousarray(v, dtype=np.int32)).to(dev) for v in (Y, X, sub))
out = torch.empty(len(Y) * len(X), dtype=torch.int32, device=dev)
st = torch.cuda.current_stream()
ts = []
for i in range(8):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    eng.fill_full_dev(y.data_ptr(), len(Y), x.data_ptr(), len(X), s.data_ptr(), 25, -11, out.data_ptr(), st.cuda_stream)
    e1.record(); torch.cuda.synchronize(); eng.sync(st.cuda_stream)
    ts.append(e0.elapsed_time(e1))
print(json.dumps({"lib": os.path.basename(os.environ["GSA_LIB"]), "ms_median": round(float(np.median(ts[2:])), 4), "last": int(out[-1])}))
PY
  done
done
