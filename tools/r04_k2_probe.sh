#!/bin/bash
# NW-LG score at K = 4 (int8) vs K = 2 (int16), and the sparse headline at K = 4 / K = 2 with both
# profile widths (GSA_KROW_K, GSA_KROW_Q8), same box.
set -e
mkdir -p gpurun_out
for r in 1 2; do
  for v in "4 1" "2 0"; do
    set -- $v
    GSA_SCORE_K=$1 GSA_KROW_Q8=$2 NO_CPU=1 timeout -k 10 200 python -u tools/score_bench.py 12000 50000 100000 > gpurun_out/nl_$1.log 2>&1
    python -c "
import json
for l in open('gpurun_out/nl_$1.log'):
    if l.startswith('{'):
        j = json.loads(l)
        if j['config'] == 'NW-LG': print('K=$1 q8=$2', j['R'], j['kernel_ms'], j['gcups'])
"
  done
done
for v in "4 1" "2 0" "2 1"; do
  set -- $v
  GSA_KROW_K=$1 GSA_KROW_Q8=$2 timeout -k 10 120 python -u bench.py --steps 10 --no-10k --no-config5 --no-cpu-baseline --config4-pairs 0 --full-batch-pairs 0 --no-rank-share 2>/dev/null | python -c "import json,sys; j=json.loads(sys.stdin.read()); print('headline K=$1 q8=$2', j['ms_per_step'], j['value'], j['golden_match'])"
done
