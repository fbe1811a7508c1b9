#!/bin/bash
# skewed K-rows kernel: parity tests of every sparse geometry, then A/B on the headline pair and shapes
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/${1:-skew}
mkdir -p $OUT; cd $ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_sparse_kernels.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -5 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/sparse_ab.py --variants ${VARIANTS:-krow:4:4:1,krow:4:4:2,krow:4:2:2,krow:4:4:1,krow:4:4:2} --reps 10 > $OUT/ab.jsonl 2>&1
rc=$?; cat $OUT/ab.jsonl; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/sparse_ab.py --variants krow:4:4:1,krow:4:4:2,krow:4:2:2 --reps 5 --shapes 1024x100000,8192x100000 > $OUT/ab_shapes.jsonl 2>&1
rc=$?; cat $OUT/ab_shapes.jsonl; exit $rc
