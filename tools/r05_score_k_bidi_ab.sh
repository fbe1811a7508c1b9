#!/bin/bash
# config 5 from both ends at 2 rows per lane (default) and 4 (GSA_SCORE_K=4), alternated.
ROOT=${GRAFT_REPO_ROOT}
O=$ROOT/gpurun_out/k4ab; mkdir -p $O
for rep in 1 2; do
  for k in default 4; do
    if [ $k = default ]; then unset GSA_SCORE_K; else export GSA_SCORE_K=$k; fi
    timeout -k 10 200 python3 $ROOT/bench.py --steps 5 --warmup 1 --no-10k --config4-pairs 0 --full-batch-pairs 0 --no-rank-share --no-cpu-baseline > $O/b_${k}_${rep}.json 2> $O/b_${k}_${rep}.err || exit 1
    python3 -c "import json; d=json.load(open('$O/b_${k}_${rep}.json'))['config5']['modes']; print('K=$k rep=$rep', {k: (m['value'], m['kernel_ms'], m['golden_match']) for k, m in d.items()})"
  done
done
