#!/bin/bash
# Score kernel with 2 rows per lane (GSA_SCORE_K=2): parity, then config 5 with K = 4 vs 2, alternated.
set -e
mkdir -p gpurun_out
GSA_SCORE_K=2 timeout -k 10 400 python -u -m pytest tests/test_gpu_score.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/score_k2.log 2>&1 || { tail -30 gpurun_out/score_k2.log; exit 1; }
echo "K=2: $(tail -1 gpurun_out/score_k2.log)"
for r in 1 2; do
  for k in 4 2; do
    GSA_SCORE_K=$k timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-10k --config4-pairs 0 --full-batch-pairs 0 --no-rank-share 2>/dev/null | python -c "import json,sys; j=json.loads(sys.stdin.read()); m=j['config5']['modes']; print('K', $k, {n: (v['kernel_ms'], v['value'], v['golden_match']) for n, v in m.items()})"
  done
done
