#!/bin/bash
# A/B of diagnostic library builds (gpuseqalign_amd/libgsa_<name>.so, tools/build_patch_variant.sh)
# against the current libgsa.so on the headline pair and a one-ticket shape: LIBS="cur a b" (each
# run twice, interleaved), optional STAMPS=<name> (a krow_stamps2 build) for tools/kr_stamps2.py.
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/${1:-ab}
mkdir -p $OUT; cd $ROOT
for rep in 1 2; do
  for lib in ${LIBS:-cur}; do
    L=$ROOT/gpuseqalign_amd/libgsa.so; [ $lib != cur ] && L=$ROOT/gpuseqalign_amd/libgsa_$lib.so
    GSA_LIB=$L timeout -k 10 200 python tools/sparse_ab.py --variants ${VARIANTS:-krow:4:4} --reps ${REPS:-6} --shapes ${SHAPES:-1024x100000,config3} > $OUT/ab_${lib}_$rep.jsonl 2>&1
    rc=$?; sed "s/^/$lib /" $OUT/ab_${lib}_$rep.jsonl | grep '{' | cut -c1-160; [ $rc -ne 0 ] && { tail -5 $OUT/ab_${lib}_$rep.jsonl; exit $rc; }
  done
done
for st in $STAMPS; do
  for shp in ${STAMP_SHAPES:-1024x100000 config3}; do
    GSA_LIB=$ROOT/gpuseqalign_amd/libgsa_$st.so timeout -k 10 200 python tools/kr_stamps2.py $shp > $OUT/stamps_${st}_$shp.txt 2>&1
    rc=$?; cat $OUT/stamps_${st}_$shp.txt | cut -c1-220; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
