set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06_gpu_all.log 2>&1 || { tail -40 gpurun_out/r06_gpu_all.log; exit 1; }
tail -3 gpurun_out/r06_gpu_all.log
