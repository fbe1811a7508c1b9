#!/bin/bash
# parity of a diagnostic build (VAR=name -> libgsa_<name>.so) on the sparse tests, then an A/B
# against the current library on config 3
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
O=gpurun_out/vc_${VAR}; mkdir -p $O
GSA_LIB=$PWD/gpuseqalign_amd/libgsa_${VAR}.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_sparse_kernels.py tests/test_gpu_sparse_random.py tests/test_gpu_mlsppt.py tests/test_gpu_goldens.py -k "${TESTK:-not 512}" > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
LIBS="cur ${VAR}" REPS=${REPS:-4} SHAPES=${SHAPES:-config3} bash tools/r03_ab.sh vc_${VAR}_ab
