set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_full100k.py > gpurun_out/r06_t26.log 2>&1 || { tail -30 gpurun_out/r06_t26.log; exit 1; }
tail -2 gpurun_out/r06_t26.log
for i in 1 2; do
timeout -k 10 120 python -u tools/r06_full100k.py --pair 10k --pitched --reps 20 | tail -1 | cut -c1-260
timeout -k 10 120 python -u tools/r06_full100k.py --pitched --reps 4 | tail -1 | cut -c1-200
done
