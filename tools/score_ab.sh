#!/bin/bash
# A/B of library builds on the score-only shapes: LIBS="cur a b" (gpuseqalign_amd/libgsa_<name>.so),
# each run twice, interleaved; SHAPES / MODES as tools/score_shape.py.
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/${1:-score_ab}
mkdir -p $OUT; cd $ROOT
for rep in 1 2; do
  for lib in ${LIBS:-cur}; do
    L=$ROOT/gpuseqalign_amd/libgsa.so; [ $lib != cur ] && L=$ROOT/gpuseqalign_amd/libgsa_$lib.so
    GSA_LIB=$L timeout -k 10 200 python tools/score_shape.py ${SHAPES:-1024x50000 50000x50000} > $OUT/${lib}_$rep.jsonl 2>&1
    rc=$?; sed "s/^/$lib /" $OUT/${lib}_$rep.jsonl | grep '{'; [ $rc -ne 0 ] && { tail -5 $OUT/${lib}_$rep.jsonl; exit $rc; }
  done
done
exit 0
