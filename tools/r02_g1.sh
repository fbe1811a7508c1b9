set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/g1
timeout -k 10 400 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_shard.py tests/test_gpu_goldens.py tests/test_gpu_sparse_kernels.py -m gpu > gpurun_out/g1/pytest.log 2>&1 || { tail -30 gpurun_out/g1/pytest.log; exit 1; }
tail -2 gpurun_out/g1/pytest.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/g1/bench.json 2> gpurun_out/g1/bench.err || { tail -20 gpurun_out/g1/bench.err; exit 1; }
cat gpurun_out/g1/bench.json
