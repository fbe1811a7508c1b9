#!/bin/bash
# round-4 PMC evidence of the 64-pair full batch (two-pass fill, pitched layout): kernel-trace stats,
# WRITE_SIZE, FETCH_SIZE and an SQ pass, one rocprofv3 run each; summaries per kernel (pass 1 =
# nw_krow_kernel XR instance, pass 2 = nw_expand_kernel)
set -e
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$ROOT/gpurun_out/${1:-pmcfb4}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- \
    python3 $ROOT/tools/batch_bench.py --mode full --pairs 64 --repeats 2 --warmup 1 > $O/log0.txt 2>&1
i=0
for ctr in "WRITE_SIZE" "FETCH_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $ctr -d $O/p$i -o run --output-format csv -- \
      python3 $ROOT/tools/batch_bench.py --mode full --pairs 64 --repeats 1 --warmup 0 > $O/log$i.txt 2>&1
done
python3 $ROOT/tools/pmc_summary.py $O nw_expand > $O/summary_expand.json
python3 $ROOT/tools/pmc_summary.py $O nw_krow > $O/summary_krow.json
cat $O/summary_expand.json $O/summary_krow.json
find $O/kt -name "*kernel_stats.csv" -exec cat {} \;
