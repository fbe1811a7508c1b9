# round check: every GPU test, smoke(), then the default bench line
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06_gpu_all2.log 2>&1 || { tail -40 gpurun_out/r06_gpu_all2.log; exit 1; }
tail -2 gpurun_out/r06_gpu_all2.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_smoke.log 2>&1 || { tail -20 gpurun_out/r06_smoke.log; exit 1; }
tail -1 gpurun_out/r06_smoke.log
