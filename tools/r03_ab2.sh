#!/bin/bash
# same-box A/Bs: lane-fill aligned segments (64-pair full batch) and the score strip kernel
# without / with its prologue spills (libgsa_stripold.so), config-5 50k
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
O=gpurun_out/ab2; mkdir -p $O
for rep in 1 2; do
  for lib in cur stripold; do
    L=$PWD/gpuseqalign_amd/libgsa.so; [ $lib != cur ] && L=$PWD/gpuseqalign_amd/libgsa_$lib.so
    NO_CPU=1 GSA_LIB=$L timeout -k 10 120 python tools/score_bench.py 50000 > $O/score_${lib}_$rep.jsonl 2>&1 || { tail $O/score_${lib}_$rep.jsonl; exit 1; }
    echo "$lib rep=$rep: $(grep -o '"config": "[A-Z-]*"\|"kernel_ms": [0-9.]*' $O/score_${lib}_$rep.jsonl | paste -sd' ')"
  done
  for al in 0 1; do
    GSA_LANE_ALIGN=$al timeout -k 10 120 python tools/batch_bench.py --mode full --pairs 64 --repeats 3 > $O/b64_${al}_$rep.json 2>&1 || { tail $O/b64_${al}_$rep.json; exit 1; }
    echo "align=$al rep=$rep: $(grep -o '"value": [0-9.]*' $O/b64_${al}_$rep.json)"
  done
done
LIBS="cur noprof" REPS=4 SHAPES=config3 bash tools/r03_ab.sh ab2_noprof
