# same-box A/B of config 5 (score-only, NW-AG and SW-LG) between the default build and GSA_LIB=$1 [$2 ...]
set -e
for r in 1 2; do
  for L in "" "$@"; do
    GSA_LIB=$L timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-10k --config4-pairs 0 --full-batch-pairs 0 --no-rank-share 2>/dev/null | python -c "import json,sys; j=json.loads(sys.stdin.read()); m=j['config5']['modes']; print('lib', '${L:-default}', {k: (v['kernel_ms'], v['value'], v['golden_match']) for k, v in m.items()})"
  done
done
