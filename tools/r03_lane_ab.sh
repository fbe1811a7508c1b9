#!/bin/bash
# same-box interleaved A/B of GSA_LANE_ALIGN on the 64-pair full batch (REPS rounds)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
O=gpurun_out/lane_ab; mkdir -p $O
for rep in $(seq ${REPS:-3}); do
  for al in 0 1; do
    GSA_LANE_ALIGN=$al timeout -k 10 120 python tools/batch_bench.py --mode full --pairs 64 --repeats 3 ${EXTRA} > $O/b64_${al}_$rep.json 2>&1 || { tail $O/b64_${al}_$rep.json; exit 1; }
    echo "align=$al rep=$rep: $(grep -o '"value": [0-9.]*' $O/b64_${al}_$rep.json)"
  done
done
