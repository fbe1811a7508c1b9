#!/bin/bash
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/${1:-diag}
mkdir -p $OUT; cd $ROOT
run() { timeout -k 10 ${T:-120} "$@"; rc=$?; echo "rc=$rc :: $*"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
T=200 run python -u -m pytest tests/test_gpu_errors.py -x -v --timeout 100 --timeout-method thread > $OUT/errors.log 2>&1
tail -5 $OUT/errors.log
for n in 256 512; do
  run python tools/batch_bench.py --pairs $n --tileBx 256 --repeats 2 --warmup 1 >> $OUT/batch.jsonl 2>> $OUT/batch.err
done
cat $OUT/batch.jsonl; grep -i error $OUT/batch.err | head -3
T=400 run python -u -m pytest tests/test_gpu_goldens.py -x -v --timeout 300 --timeout-method thread > $OUT/goldens.log 2>&1
tail -8 $OUT/goldens.log
