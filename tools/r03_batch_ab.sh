#!/bin/bash
# full-batch (64 x 20k) and 10k single-pair A/B of LIBS ("cur name ..."), interleaved
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
O=gpurun_out/${1:-batch_ab}; mkdir -p $O
for rep in $(seq ${REPS:-3}); do
  for lib in ${LIBS:-cur}; do
    L=$PWD/gpuseqalign_amd/libgsa.so; [ $lib != cur ] && L=$PWD/gpuseqalign_amd/libgsa_$lib.so
    GSA_LIB=$L timeout -k 10 120 python tools/batch_bench.py --mode full --pairs 64 --repeats 3 > $O/b64_${lib}_$rep.json 2>&1 || { tail $O/b64_${lib}_$rep.json; exit 1; }
    GSA_LIB=$L timeout -k 10 120 python tools/batch_bench.py --mode full --pairs 1 --lo 10000 --hi 10000 --repeats 10 > $O/b1_${lib}_$rep.json 2>&1 || { tail $O/b1_${lib}_$rep.json; exit 1; }
    echo "$lib rep=$rep 64x20k: $(grep -o '"value": [0-9.]*' $O/b64_${lib}_$rep.json) 10k: $(grep -o '"value": [0-9.]*' $O/b1_${lib}_$rep.json)"
  done
done
