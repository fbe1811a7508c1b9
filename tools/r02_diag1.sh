#!/bin/bash
# diagnostics: headline bench without config4, then batch sizes; stop on any abnormal exit
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/${1:-diag}
mkdir -p $OUT; cd $ROOT
run() { timeout -k 10 ${T:-120} "$@"; rc=$?; echo "rc=$rc :: $*"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
T=300 run python bench.py --config4-pairs 0 --cpu-budget 6 > $OUT/bench_nocfg4.json 2> $OUT/bench_nocfg4.err
cat $OUT/bench_nocfg4.json; tail -3 $OUT/bench_nocfg4.err
for tb in 512 256; do for n in 64 128 256 512; do
  run python tools/batch_bench.py --pairs $n --tileBx $tb --repeats 2 --warmup 1 >> $OUT/batch.jsonl 2>> $OUT/batch.err
done; done
cat $OUT/batch.jsonl; grep -i error $OUT/batch.err | head
