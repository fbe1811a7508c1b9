#!/bin/bash
# K-rows sparse kernel breakdown: block stamps (stamp build) and knob ablation (timing builds).
# Stops on any abnormal exit.
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/${1:-diag3}
mkdir -p $OUT; cd $ROOT
run() { timeout -k 10 ${T:-120} "$@"; rc=$?; echo "rc=$rc :: $*"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
GSA_LIB=$ROOT/gpuseqalign_amd/libgsa_p2stamp.so run python tools/kr_stamps.py 1024 100000 > $OUT/stamps_1024.txt 2>&1
GSA_LIB=$ROOT/gpuseqalign_amd/libgsa_p2stamp.so run python tools/kr_stamps.py 8192 100000 > $OUT/stamps_8192.txt 2>&1
cat $OUT/stamps_1024.txt $OUT/stamps_8192.txt | grep strip
SHAPES=1024x100000,8192x100000,100000x100000 bash tools/r02_knobs.sh diag3/knobs 1 4 8 16 32 9
