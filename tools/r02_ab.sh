#!/bin/bash
# A/B of the current libgsa against libgsa_base.so (the previous build): sparse parity tests of the
# current build first, then tools/sparse_ab.py on the headline pair and two random shapes.
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/${1:-ab}
mkdir -p $OUT; cd $ROOT
timeout -k 10 300 python -u -m pytest ${TESTS:-tests/test_gpu_sparse_kernels.py tests/test_gpu_goldens.py} -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -5 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
for lib in base cur base cur; do
  L=$ROOT/gpuseqalign_amd/libgsa.so; [ $lib = base ] && L=$ROOT/gpuseqalign_amd/libgsa_base.so
  GSA_LIB=$L timeout -k 10 200 python tools/sparse_ab.py --variants ${VARIANTS:-krow:4:4} --reps 10 --shapes ${SHAPES:-1024x100000,config3} > $OUT/ab_$lib.jsonl 2>&1
  rc=$?; sed "s/^/$lib /" $OUT/ab_$lib.jsonl | grep '{'; [ $rc -ne 0 ] && exit $rc
done
exit 0
