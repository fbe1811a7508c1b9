#!/bin/bash
# config 5 (50k x 50k score-only SW-LG and NW-AG, bench.py config5) with SW from both ends (default)
# and without it (GSA_SCORE_BIDI_SW=0), alternated, each in its own process.
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$ROOT/gpurun_out/${1:-swb}; mkdir -p $O
for rep in 1 2; do
  for v in 1 0; do
    GSA_SCORE_BIDI_SW=$v timeout -k 10 200 python3 $ROOT/bench.py --steps 5 --warmup 1 --no-10k --config4-pairs 0 \
        --full-batch-pairs 0 --no-rank-share --no-cpu-baseline > $O/b_${v}_${rep}.json 2> $O/b_${v}_${rep}.err || exit 1
    python3 -c "import json; d=json.load(open('$O/b_${v}_${rep}.json'))['config5']['modes']; print('bidi_sw=$v rep=$rep', {k: (m['value'], m['kernel_ms'], m['golden_match']) for k, m in d.items()})"
  done
done
