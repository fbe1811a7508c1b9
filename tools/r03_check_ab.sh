#!/bin/bash
# Parity first (sparse kernels, goldens, laps), then A/B timing of LIBS and stamp builds (tools/r03_ab.sh).
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/${1:-chk}
mkdir -p $OUT; cd $ROOT
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_sparse_kernels.py tests/test_gpu_goldens.py tests/test_gpu_parity.py} -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && { tail -30 $OUT/pytest.log; exit $rc; }
bash tools/r03_ab.sh ${1:-chk}
