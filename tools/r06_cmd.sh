set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
LIBS="ffp" bash tools/r06_ab.sh
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06_gpu_all4.log 2>&1
tail -2 gpurun_out/r06_gpu_all4.log
for i in 1 2; do
timeout -k 10 120 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --config4-pairs 0 --no-10k --no-100k-full --no-rank-share --full-batch-pairs 0 --no-config5 2>/dev/null | grep '^{' | python3 -c "import sys,json; j=json.loads(sys.stdin.read()); print('headline', j['value'], j['ms_per_step'], j['roofline']['kernel_ms'])"
done
