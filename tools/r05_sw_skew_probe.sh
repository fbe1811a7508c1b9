#!/bin/bash
# SW-LG / SW-AG 50k from both ends (bench.py config5) under GSA_BIDI_SKEW (rows the top half takes past
# R/2; unset = the cost model), each setting in its own process.
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$ROOT/gpurun_out/swskew; mkdir -p $O
for sk in ${SKEWS:-model 0 800 2500 3500}; do
  if [ $sk = model ]; then unset GSA_BIDI_SKEW; else export GSA_BIDI_SKEW=$sk; fi
  timeout -k 10 200 python3 $ROOT/bench.py --steps 5 --warmup 1 --no-10k --config4-pairs 0 --full-batch-pairs 0 \
      --no-rank-share --no-cpu-baseline > $O/b_$sk.json 2> $O/b_$sk.err || exit 1
  python3 -c "import json; d=json.load(open('$O/b_$sk.json'))['config5']['modes']; print('skew=$sk', {k: (m['value'], m['kernel_ms'], m['golden_match']) for k, m in d.items()})"
done
