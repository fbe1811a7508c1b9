#!/bin/bash
# aligned-segment lane variant (libgsa_al.so) vs current on the full batch: same-box A/B, then the
# PMC WRITE_SIZE of one launch of each
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $ROOT
LIBS="cur al" REPS=3 bash tools/r03_batch_ab.sh al_ab || exit 1
cd /tmp && export TMPDIR=/tmp
for lib in cur al; do
  L=$ROOT/gpuseqalign_amd/libgsa.so; [ $lib != cur ] && L=$ROOT/gpuseqalign_amd/libgsa_$lib.so
  O=$ROOT/gpurun_out/al_pmc_$lib; mkdir -p $O
  GSA_LIB=$L timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d $O/p1 -o run --output-format csv -- \
      python3 $ROOT/tools/batch_bench.py --mode full --pairs 64 --repeats 1 --warmup 0 > $O/log1.txt 2>&1 || exit 1
  python3 $ROOT/tools/pmc_summary.py $O nw_lane > $O/summary.json
  echo "$lib $(cat $O/summary.json | tr -d '\n ')"
done
