#!/bin/bash
# knob ablation of a sparse kernel build family (KPFX: libgsa_<KPFX><bits>.so; timing only); stops on any abnormal exit
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/${1:-knobs}; shift
mkdir -p $OUT; cd $ROOT
for k in "" "$@"; do
  lib=$ROOT/gpuseqalign_amd/libgsa${k:+_${KPFX:-krk}$k}.so
  GSA_LIB=$lib timeout -k 10 120 python tools/sparse_ab.py --variants ${VARIANT:-krow:4:4} --reps 5 --shapes ${SHAPES:-1024x100000,8192x100000} > $OUT/k$k.jsonl 2>&1
  rc=$?; echo "knob '$k' rc=$rc"; grep '^{' $OUT/k$k.jsonl | sed "s/^/k$k /"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
