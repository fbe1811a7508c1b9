#!/bin/bash
# Full batch variants on one box, each in its own process: one group (default), the split groups
# (GSA_FULL_SPLIT=1), and a persistent 16-wave expansion (GSA_EXPAND_GRID=256).
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$ROOT/gpurun_out/${1:-split}; mkdir -p $O
for rep in 1 2; do
  for v in "GSA_FULL_SPLIT=0" "GSA_FULL_SPLIT=1" "GSA_EXPAND_GRID=256" "GSA_EXPAND_GRID=512"; do
    env $v timeout -k 10 200 python3 $ROOT/bench.py --steps 3 --warmup 1 --no-10k --no-config5 \
        --config4-pairs 0 --no-cpu-baseline > $O/b.json 2> $O/b.err || exit 1
    python3 -c "import json; d=json.load(open('$O/b.json'))['full_batch']; p=d['passes']; print('$v rep=$rep', d['value'], d['hbm_frac'], d['seconds'], p.get('pass1_ms'), p.get('pass2_ms'), d['pairs_matching_golden'])"
  done
done
