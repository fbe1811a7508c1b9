set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "full or fused or twopass or expansion or split" > gpurun_out/r06_t27.log 2>&1 || { tail -30 gpurun_out/r06_t27.log; exit 1; }
tail -1 gpurun_out/r06_t27.log
LIBS="whole" bash tools/r06_ab.sh
