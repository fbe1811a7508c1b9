#!/bin/bash
# Score fix + grouped two-pass parity, then the 64-pair full batch with GSA_FULL_GROUPS 1 / 2 / 4,
# alternated twice (same box).
set -e
timeout -k 10 500 python -u -m pytest tests/test_gpu_score.py tests/test_gpu_sparse_kernels.py tests/test_gpu_parity.py -k "score or sparse or twopass_tables" -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/groups_tests.log 2>&1 || { tail -30 gpurun_out/groups_tests.log; exit 1; }
tail -1 gpurun_out/groups_tests.log
for r in 1 2; do
  for g in 1 2 4; do
    GSA_FULL_GROUPS=$g timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-10k --no-config5 --no-cpu-baseline --config4-pairs 0 --no-rank-share 2>/dev/null | python -c "import json,sys; j=json.loads(sys.stdin.read()); f=j['full_batch']; print('groups', $g, f['value'], f['seconds'], f['hbm_frac'])"
  done
done
