#!/bin/bash
# One GPU session: parity suite, smoke, bench (JSON line), then rocprofv3 kernel traces of the bench
# in isolated passes (tools/r05_prof.sh: the headline alone, then the other fields without the rank
# shares, so every roofline input is one row of its own) and the headline's PMC pass.
# Each GPU step has its own time limit; the first failure ends the script.
set -e
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-check}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
bash $ROOT/tools/r05_prof.sh $TAG/prof > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
tail -4 $OUT/prof.log
