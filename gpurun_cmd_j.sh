mkdir -p gpurun_out/r03_j
timeout -k 10 400 python -u -m pytest tests/test_gpu_sparse_kernels.py tests/test_gpu_goldens.py tests/test_gpu_mlsppt.py tests/test_gpu_laps.py tests/test_gpu_sparse_random.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r03_j/pytest.log 2>&1; tail -2 gpurun_out/r03_j/pytest.log
REPS=5 LIBS="cur base" bash tools/r03_ab.sh r03_j
GSA_PT_DEBUG=1 timeout -k 10 300 python tools/mlsppt_bench.py 5 > gpurun_out/r03_j/mlsppt.jsonl 2>&1; tail -12 gpurun_out/r03_j/mlsppt.jsonl | cut -c1-200
