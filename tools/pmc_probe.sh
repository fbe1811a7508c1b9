#!/bin/bash
# PMC passes (one counter group per pass, no trace domains) over one fill configuration.
# usage: tools/pmc_probe.sh OUTDIR R C MODE [TILEBX]
set -e
OUT=$1; R=$2; C=$3; MODE=$4; TBX=${5:-256}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd /tmp && export TMPDIR=/tmp
mkdir -p $ROOT/$OUT
i=0
for ctr in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_WR" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $ctr -d $ROOT/$OUT/p$i -o run --output-format csv -- \
      python3 $ROOT/tools/prof_one.py --R $R --C $C --mode $MODE --tileBx $TBX --reps 2 > $ROOT/$OUT/log$i.txt 2>&1
done
