#!/bin/bash
# pass-2 PMC, default tasks vs 4 tiles per wave per task (GSA_EXPAND_MT=4): kernel time, wave cycles,
# waits, occupancy (64-pair full batch, one launch each)
set -e
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd /tmp && export TMPDIR=/tmp
for mt in 1 4; do
  O=$ROOT/gpurun_out/pmcmt$mt; mkdir -p $O
  GSA_EXPAND_MT=$mt timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/p1 -o run --output-format csv -- \
      python3 $ROOT/tools/batch_bench.py --mode full --pairs 64 --repeats 1 --warmup 0 > $O/log1.txt 2>&1
  python3 $ROOT/tools/pmc_summary.py $O nw_expand > $O/summary.json
  echo "mt $mt"; cat $O/summary.json
done
