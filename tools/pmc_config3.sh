#!/bin/bash
# PMC passes (one counter group per pass, no trace domains) over the bench's headline fill
# (BASELINE configs[2]); a kernel-trace --stats pass of the same program first.
# usage: tools/pmc_config3.sh OUTDIR
set -e
OUT=$1
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd /tmp && export TMPDIR=/tmp
mkdir -p $ROOT/$OUT
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/kt -o run --output-format csv -- \
    python3 $ROOT/tools/prof_one.py --config3 --reps 5 > $ROOT/$OUT/log0.txt 2>&1
i=0
for ctr in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_WR" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
           "GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVES SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctr -d $ROOT/$OUT/p$i -o run --output-format csv -- \
      python3 $ROOT/tools/prof_one.py --config3 --reps 2 > $ROOT/$OUT/log$i.txt 2>&1
done
