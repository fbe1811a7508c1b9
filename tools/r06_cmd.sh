set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06_gpu_all3.log 2>&1
tail -3 gpurun_out/r06_gpu_all3.log
timeout -k 10 120 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --config4-pairs 0 --no-10k --no-100k-full --no-rank-share --full-batch-pairs 0 --no-config5 2>/dev/null | grep '^{' > gpurun_out/r06_hl.json
python3 -c "import json; j=json.load(open('gpurun_out/r06_hl.json')); print(j['value'], j['ms_per_step'], j['roofline']['kernel_ms'])"
