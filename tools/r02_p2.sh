#!/bin/bash
# pair2 bring-up: sparse parity tests, then an A/B of the single-pair sparse kernels
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/${1:-p2}
mkdir -p $OUT; cd $ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_goldens.py tests/test_gpu_check.py tests/test_gpu_trace.py -x -v --timeout 300 --timeout-method thread -k "sparse or config3 or trace or check" > $OUT/pytest.log 2>&1
rc=$?; tail -15 $OUT/pytest.log; echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/sparse_ab.py > $OUT/ab.jsonl 2> $OUT/ab.err; rc=$?
cat $OUT/ab.jsonl; tail -3 $OUT/ab.err; exit $rc
