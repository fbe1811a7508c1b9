set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_score.py -k "both_ends_100k or large_random" --durations=5 > gpurun_out/r06_t28.log 2>&1 || { tail -30 gpurun_out/r06_t28.log; exit 1; }
tail -12 gpurun_out/r06_t28.log
