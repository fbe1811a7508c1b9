#!/bin/bash
# Full batch (bench.py full_batch: 64 x 18-22k, 102 GB) in one group (GSA_FULL_SPLIT=0), split in
# two groups (1) and tuned (unset: the four candidates timed on the first launches, GSA_TUNE_LOG
# prints their times), interleaved, each in its own process.
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$ROOT/gpurun_out/${1:-split}; mkdir -p $O
for rep in 1 2; do
  for sp in 0 1 tuned; do
    if [ $sp = tuned ]; then unset GSA_FULL_SPLIT; else export GSA_FULL_SPLIT=$sp; fi
    GSA_TUNE_LOG=1 timeout -k 10 200 python3 $ROOT/bench.py --steps 3 --warmup 1 --no-10k --no-config5 \
        --config4-pairs 0 --no-cpu-baseline > $O/b_${sp}_${rep}.json 2> $O/b_${sp}_${rep}.err || exit 1
    grep "full-batch tuning" $O/b_${sp}_${rep}.err || true
    python3 -c "import json; d=json.load(open('$O/b_${sp}_${rep}.json'))['full_batch']; p=d['passes']; print('split=$sp rep=$rep', d['value'], d['hbm_frac'], d['seconds'], p.get('pass1_ms'), p.get('pass2_ms'), p.get('pipelined_groups'), d['pairs_matching_golden'])"
  done
done
