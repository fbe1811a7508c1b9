#!/bin/bash
# Score kernel int8-profile check: parity tests, then config5 with the int16 profile vs the int8 one.
set -e
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/ksq8
mkdir -p $OUT
cd $ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_score.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for q in 0 1 0 1; do
  GSA_KROW_Q8=$q timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-10k --config4-pairs 0 --full-batch-pairs 0 --no-rank-share > $OUT/b$q.json 2> $OUT/b$q.err || { tail -20 $OUT/b$q.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/b$q.json'));m=d['config5']['modes'];print('q8=$q',{k: (v['kernel_ms'], v['value'], v['golden_match']) for k, v in m.items()})"
done
