#!/bin/bash
# round 5: process-to-process variance of the full batch: 8 bench processes (full batch field only,
# two launches), alternating a 16 GiB fill before the batch (GSA_BENCH_FILL_FIRST=1) and none
set -e
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $ROOT
for r in 1 2 3 4; do
  for F in 0 1; do
    GSA_FULL_PIPE=0 GSA_BENCH_FILL_FIRST=$F timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-10k --no-config5 \
        --no-cpu-baseline --config4-pairs 0 --no-rank-share 2>/dev/null | python -c "
import json,sys; j=json.loads(sys.stdin.read()); f=j['full_batch']; p=f['passes']
print('fill_first $F', 'batch_s', f['seconds'], 'p1', p['pass1_ms'], 'p2', p['pass2_ms'], 'clk', p['clock_ghz_median'], 'box', f['box_fill'])"
  done
done
