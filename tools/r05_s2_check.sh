#!/bin/bash
# round 5: the SYNC2 strip build (GSA_KROW_SYNC2=1: check/halo/hand-off every 32 steps) -- sparse
# parity tests through it, then the bench (headline, 10k, config 4, full batch) against the default
# build, alternated 3 times
set -e
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$ROOT/gpurun_out/${1:-r05s2}; mkdir -p $O
cd $ROOT
GSA_LIB=$ROOT/gpuseqalign_amd/libgsa_s2.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_goldens.py -x -q \
    --timeout 120 --timeout-method thread > $O/pytest_s2.log 2>&1 || { tail -30 $O/pytest_s2.log; exit 1; }
tail -2 $O/pytest_s2.log
for r in 1 2 3; do
  for L in "" "$ROOT/gpuseqalign_amd/libgsa_s2.so"; do
    GSA_LIB=$L timeout -k 10 300 python -u bench.py --steps 20 --no-config5 --no-cpu-baseline --no-rank-share --full-batch-pairs 0 2>>$O/bench.err | python -c "
import json,sys; j=json.loads(sys.stdin.read())
print('lib', '${L:-default}'.split('/')[-1], 'headline_ms', j['roofline']['kernel_ms'], 'gcups', j['value'], 'gold', j['golden_match'], '10k_ms', j['fill_10k_full']['kernel_ms'], 'cfg4_s', j['config4']['seconds'], j['config4']['pairs_matching_golden'])" | tee -a $O/ab.txt
  done
done
