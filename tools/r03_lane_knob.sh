#!/bin/bash
# lane fill A/B: aligned segments on/off, with and without output stores (libgsa_nostore.so),
# on the 64-pair full batch and one 10k pair
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
O=gpurun_out/lane_knob; mkdir -p $O
for lib in cur nostore; do
  L=$PWD/gpuseqalign_amd/libgsa.so; [ $lib != cur ] && L=$PWD/gpuseqalign_amd/libgsa_$lib.so
  for al in 0 1; do
    GSA_LIB=$L GSA_LANE_ALIGN=$al timeout -k 10 120 python tools/batch_bench.py --mode full --pairs 64 --repeats 3 > $O/b64_${lib}_$al.json 2>&1 || { tail $O/b64_${lib}_$al.json; exit 1; }
    GSA_LIB=$L GSA_LANE_ALIGN=$al timeout -k 10 120 python tools/batch_bench.py --mode full --pairs 1 --lo 10000 --hi 10000 --repeats 10 > $O/b1_${lib}_$al.json 2>&1 || { tail $O/b1_${lib}_$al.json; exit 1; }
    echo "$lib align=$al 64x20k: $(grep -o '"value": [0-9.]*' $O/b64_${lib}_$al.json)  10k: $(grep -o '"value": [0-9.]*' $O/b1_${lib}_$al.json)"
  done
done
