#!/bin/bash
# score-mode parity, then config-5 kernel times of LIBS ("cur name ...") interleaved
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
O=gpurun_out/${1:-score_ab}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_score.py tests/test_gpu_laps.py > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
for rep in $(seq ${REPS:-3}); do
  for lib in ${LIBS:-cur}; do
    L=$PWD/gpuseqalign_amd/libgsa.so; [ $lib != cur ] && L=$PWD/gpuseqalign_amd/libgsa_$lib.so
    NO_CPU=1 GSA_LIB=$L timeout -k 10 120 python tools/score_bench.py 50000 > $O/score_${lib}_$rep.jsonl 2>&1 || { tail $O/score_${lib}_$rep.jsonl; exit 1; }
    echo "$lib rep=$rep: $(grep -o '"config": "[A-Z-]*"\|"kernel_ms": [0-9.]*' $O/score_${lib}_$rep.jsonl | paste -sd' ')"
  done
done
