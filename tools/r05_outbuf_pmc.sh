#!/bin/bash
# PMC passes over the full batch's pass 2 in its slow state (the process's first 102 GB output
# buffer) and its fast one (the buffer allocated again after torch.cuda.empty_cache()):
# tools/r05_outbuf_probe.py pmc, one pass per counter group.  usage: tools/r05_outbuf_pmc.sh TAG
set -e
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$ROOT/gpurun_out/${1:-obufpmc}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for ctr in "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_THRASHING_STALL_sum" \
           "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum GRBM_GUI_ACTIVE" \
           "TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum TCP_UTCL1_SERIALIZATION_STALL_sum TCP_TCC_WRITE_REQ_LATENCY_sum TCP_TCC_WRITE_REQ_sum"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $ctr -d $O/p$i -o run --output-format csv -- \
      python3 $ROOT/tools/r05_outbuf_probe.py pmc > $O/log$i.txt 2>&1
done
