#!/bin/bash
# round 5: the pipelined full batch -- its parity tests, then the bench's full-batch field with
# 2 / 4 / 8 groups and the two-launch path (GSA_FULL_PIPE=0), alternated twice
set -e
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$ROOT/gpurun_out/${1:-r05pipe}; mkdir -p $O
cd $ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread \
    -k "pipelined or twopass_tables or full_timing" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 120 ./tools/ubench/lds_gran_probe > $O/lds_gran.txt 2>&1 || true
for r in 1 2; do
  for P in 0 2 4 8; do
    GSA_FULL_PIPE=$P timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-10k --no-config5 --no-cpu-baseline \
        --config4-pairs 0 --no-rank-share 2>>$O/bench.err | python -c "
import json,sys; j=json.loads(sys.stdin.read()); f=j['full_batch']; p=f['passes']
print('pipe', $P, 'batch_s', f['seconds'], 'gcups', f['value'], 'hbm_frac', f['hbm_frac'], 'p1', p['pass1_ms'], 'p2', p['pass2_ms'], 'clk', p['clock_ghz_median'], 'gold', f['pairs_matching_golden'])" | tee -a $O/ab.txt
  done
done
