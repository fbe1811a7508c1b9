# same-box A/B of the headline (configs[2] only) between the default build and diagnostic builds
# (GSA_LIB=$1 [$2 ...]), alternated 3 times
set -e
mkdir -p gpurun_out
for r in 1 2 3; do
  for L in "" "$@"; do
    GSA_LIB=$L timeout -k 10 120 python -u bench.py --steps 20 --no-10k --no-config5 --no-cpu-baseline --config4-pairs 0 --full-batch-pairs 0 --no-rank-share 2>/dev/null | python -c "import json,sys; j=json.loads(sys.stdin.read()); print('lib', '${L:-default}', j['ms_per_step'], j['value'], j['roofline']['kernel_ms'])"
  done
done
