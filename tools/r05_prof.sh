#!/bin/bash
# Round-5 rocprof evidence with each roofline input on a row of its own:
#   A: the bench with the headline alone  -> nw_krow_kernel<4,4,1024,0,true> = configs[2] only
#   B: the bench without the rank shares  -> nw_krow_kernel<8,4,1024,0,true> = config 4 only,
#      nw_krow_kernel<8,4,1024,2,true> + nw_expand_kernel<16> = the full batch's two passes,
#      nw_full_fused_kernel<4,8,true> = configs[1]
#   C: config 5 with a short headline -> nw_kscore_kernel<3,false,2> (NW-AG, both halves in one
#      launch) and <5,false,2> (SW-LG)
#   PMC passes over the headline fill alone (tools/prof_one.py --config3): SQ instruction mix per
#   dispatch (SQ_INSTS_SALU / _VALU / _LDS), waves, cycles, GRBM_GUI_ACTIVE (clock)
# usage: tools/r05_prof.sh TAG  (outputs under gpurun_out/TAG)
set -e
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$ROOT/gpurun_out/${1:-r05prof}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/A -o run --output-format csv -- \
    python3 $ROOT/bench.py --steps 20 --warmup 3 --no-10k --no-config5 --config4-pairs 0 --full-batch-pairs 0 \
    --no-cpu-baseline > $O/A_bench.json 2> $O/A.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/B -o run --output-format csv -- \
    python3 $ROOT/bench.py --steps 20 --warmup 3 --no-config5 --no-rank-share --no-cpu-baseline \
    > $O/B_bench.json 2> $O/B.err
# C: config 5 (score-only 50k NW-AG from both ends, SW-LG) beside a short headline run
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/C -o run --output-format csv -- \
    python3 $ROOT/bench.py --steps 8 --warmup 2 --no-10k --config4-pairs 0 --full-batch-pairs 0 \
    --no-cpu-baseline > $O/C_bench.json 2> $O/C.err
i=0
for ctr in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU" \
           "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctr -d $O/p$i -o run --output-format csv -- \
      python3 $ROOT/tools/prof_one.py --config3 --reps 2 > $O/log$i.txt 2>&1
done
python3 $ROOT/tools/pmc_summary.py $O "nw_krow_kernel<4, 4, 1024, 0, true>" > $O/pmc_headline.json
cat $O/pmc_headline.json
find $O/A $O/B $O/C -name "*kernel_stats.csv" | sort
