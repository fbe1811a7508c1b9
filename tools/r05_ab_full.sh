#!/bin/bash
# same-box A/B of the full batch (bench full_batch field: both passes' HIP-event times and pass 2's
# effective clock) between the default build and GSA_LIB=$1 [$2 ...], alternated 3 times
set -e
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $ROOT
for r in 1 2 3; do
  for L in "" "$@"; do
    GSA_LIB=$L timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-10k --no-config5 --no-cpu-baseline \
        --config4-pairs 0 --no-rank-share 2>/dev/null | python -c "
import json,sys; j=json.loads(sys.stdin.read()); f=j['full_batch']; p=f['passes']
print('lib', '${L:-default}', 'batch_s', f['seconds'], 'gcups', f['value'], 'hbm_frac', f['hbm_frac'], 'p1', p['pass1_ms'], 'p2', p['pass2_ms'], 'clk', p['clock_ghz_median'], 'box', (f.get('box_fill') or {}).get('GBps'), 'gold', f['pairs_matching_golden'])"
  done
done
