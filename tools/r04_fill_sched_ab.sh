#!/bin/bash
# same-box A/B of the default build against GSA_LIB=$1 on the 10k fused full fill and the 64-pair
# full batch (bench fields), alternated twice
set -e
for r in 1 2; do
  for L in "" "$@"; do
    GSA_LIB=$L timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-config5 --no-cpu-baseline --config4-pairs 0 --no-rank-share 2>/dev/null | python -c "import json,sys; j=json.loads(sys.stdin.read()); print('lib', '${L:-default}', 'headline', j['ms_per_step'], '10k', j['fill_10k_full']['kernel_ms'], j['fill_10k_full']['value'], 'batch', j['full_batch']['seconds'], j['full_batch']['value'])"
  done
done
