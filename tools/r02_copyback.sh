# host-buffer copy-back through pinned chunks on 4 threads: parity of the host-buffer paths, then mlsp / mlsppt end to end
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/cb; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_mlsppt.py tests/test_gpu_sparse_kernels.py tests/test_gpu_goldens.py tests/test_host_cli.py tests/test_capi.py -m gpu > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python tools/verify_bench.py > $O/verify.jsonl 2> $O/verify.err || { tail -20 $O/verify.err; exit 1; }
grep mlsp $O/verify.jsonl
