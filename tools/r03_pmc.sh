#!/bin/bash
# round-3 PMC evidence: the headline fill (tools/pmc_config3.sh) and the 64-pair full batch
# (kernel-trace stats + WRITE_SIZE + FETCH_SIZE, one pass each)
set -e
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
bash $ROOT/tools/pmc_config3.sh gpurun_out/pmc3
cd /tmp && export TMPDIR=/tmp
O=$ROOT/gpurun_out/pmcfb; mkdir -p $O
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- \
    python3 $ROOT/tools/batch_bench.py --mode full --pairs 64 --repeats 2 --warmup 1 > $O/log0.txt 2>&1
i=0
for ctr in "WRITE_SIZE" "FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $ctr -d $O/p$i -o run --output-format csv -- \
      python3 $ROOT/tools/batch_bench.py --mode full --pairs 64 --repeats 1 --warmup 0 > $O/log$i.txt 2>&1
done
python3 $ROOT/tools/pmc_summary.py $ROOT/gpurun_out/pmc3 nw_krow > $ROOT/gpurun_out/pmc3/summary.json
python3 $ROOT/tools/pmc_summary.py $O nw_lane > $O/summary.json
cat $ROOT/gpurun_out/pmc3/summary.json $O/summary.json
