#!/bin/bash
# Round-6 rocprof evidence (one kernel per row):
#   A: kernel-trace --stats of the bench's headline alone -> nw_krow_kernel<4,4,1024,0,true>
#   B: kernel-trace --stats of the 100k x 100k full fill alone (pitched, fused: one launch per fill)
#      -> one homogeneous nw_full_fused_kernel<4,8,true> row
#   C: kernel-trace --stats of the 64-pair full batch (6 untimed + 3 timed launches, as the bench)
#   PMC: WRITE_SIZE and FETCH_SIZE, one pass each, over the headline, the 100k full fill and the batch
# usage: tools/r06_prof.sh TAG  (outputs under gpurun_out/TAG)
set -e
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$ROOT/gpurun_out/${1:-r06prof}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/A -o run --output-format csv -- \
    python3 $ROOT/bench.py --steps 20 --warmup 3 --no-10k --no-100k-full --no-config5 --config4-pairs 0 \
    --full-batch-pairs 0 --no-cpu-baseline > $O/A_bench.json 2> $O/A.err
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/B -o run --output-format csv -- \
    python3 $ROOT/tools/r06_full100k.py --pitched --reps 5 > $O/B.json 2> $O/B.err
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/C -o run --output-format csv -- \
    python3 $ROOT/tools/batch_bench.py --mode full --pairs 64 --warmup 6 --repeats 3 > $O/C.json 2> $O/C.err
for ctr in WRITE_SIZE FETCH_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $ctr -d $O/h_$ctr -o run --output-format csv -- \
      python3 $ROOT/tools/prof_one.py --config3 --reps 2 > $O/h_$ctr.log 2>&1
  timeout -s KILL 180 rocprofv3 --pmc $ctr -d $O/f_$ctr -o run --output-format csv -- \
      python3 $ROOT/tools/r06_full100k.py --pitched --reps 1 > $O/f_$ctr.log 2>&1
  timeout -s KILL 180 rocprofv3 --pmc $ctr -d $O/b_$ctr -o run --output-format csv -- \
      python3 $ROOT/tools/batch_bench.py --mode full --pairs 64 --warmup 0 --repeats 1 > $O/b_$ctr.log 2>&1
done
find $O -name "*kernel_stats.csv" | sort
