#!/bin/bash
# timing of several libgsa builds (LIBS: suffixes, "" = libgsa.so) on SHAPES; stops on abnormal exit
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/${1:-libs}
mkdir -p $OUT; cd $ROOT
for rep in 1 2; do
for l in $LIBS; do
  L=$ROOT/gpuseqalign_amd/libgsa$l.so; [ "$l" = "cur" ] && L=$ROOT/gpuseqalign_amd/libgsa.so
  GSA_LIB=$L timeout -k 10 200 python tools/sparse_ab.py --variants ${VARIANTS:-krow:4:4} --reps ${REPS:-5} --shapes ${SHAPES:-1024x100000,config3} > $OUT/t_$l.jsonl 2>&1
  rc=$?; python3 -c "
import json,sys
for line in open('$OUT/t_$l.jsonl'):
    if line.startswith('{'):
        d=json.loads(line); print('$l'.ljust(8), f\"{d['R']}x{d['C']}\".ljust(14), d['ms_median'], d['align_cost'], d.get('golden'))"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -3 $OUT/t_$l.jsonl; exit $rc; fi
done; done
