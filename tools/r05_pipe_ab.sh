#!/bin/bash
# round 5: full-batch variants on one box (bench full_batch field), alternated twice:
#   base (two launches, 16-wave per-task expansion), persistent 12-wave expansion, pair-major tasks,
#   the pipelined batch with 2 groups
set -e
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$ROOT/gpurun_out/${1:-r05pab}; mkdir -p $O
cd $ROOT
for r in 1 2; do
  for V in "GSA_FULL_PIPE=0" "GSA_FULL_PIPE=0 GSA_EXPAND_GRID=256 GSA_EXPAND_WAVES=12" "GSA_FULL_PIPE=0 GSA_EXPAND_RR=0" "GSA_FULL_PIPE=2" ${EXTRA}; do
    env $V timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-10k --no-config5 --no-cpu-baseline \
        --config4-pairs 0 --no-rank-share 2>>$O/bench.err | python -c "
import json,sys; j=json.loads(sys.stdin.read()); f=j['full_batch']; p=f['passes']
print('$V |', 'batch_s', f['seconds'], 'hbm_frac', f['hbm_frac'], 'p1', p['pass1_ms'], 'p2', p['pass2_ms'], 'clk', p['clock_ghz_median'], 'box', f['box_fill'].get('GBps'), 'over_box', f['over_box_fill'], 'gold', f['pairs_matching_golden'])" | tee -a $O/ab.txt
  done
done
