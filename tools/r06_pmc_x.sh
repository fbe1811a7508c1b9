#!/bin/bash
# PMC passes over the 100k x 100k full fill (pitched; $1 = GSA_FULL_FUSED value, 0 = two launches),
# one rocprofv3 run per counter group; summaries for the expansion (nw_expand) and fused kernels
set -e
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$ROOT/gpurun_out/${2:-r06pmcx}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export GSA_FULL_FUSED=${1:-0}
i=0
for ctr in "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_THRASHING_STALL_sum" \
           "WRITE_SIZE" "TA_BUSY_sum TA_DATA_STALLED_BY_TC_CYCLES_sum" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY" \
           "TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TCC_WRITE_REQ_LATENCY_sum" \
           "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $ctr -d $O/p$i -o run --output-format csv -- \
      python3 $ROOT/tools/r06_full100k.py --reps 1 --pitched > $O/log$i.txt 2>&1
done
python3 $ROOT/tools/pmc_summary.py $O "nw_expand|nw_full_fused" > $O/summary.json
cat $O/summary.json
