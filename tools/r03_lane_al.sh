#!/bin/bash
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
O=gpurun_out/lane_al; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "aligned_segments or full_kernel_shapes or lane_kernel_wide" tests/test_shard.py > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -3 $O/pytest.txt
for rep in 1 2; do
for al in 0 1; do
GSA_LANE_ALIGN=$al timeout -k 10 120 python tools/batch_bench.py --mode full --pairs 64 --repeats 3 > $O/bb_${al}_$rep.json 2>&1 || { tail $O/bb_${al}_$rep.json; exit 1; }
echo "align=$al $(cut -c1-200 $O/bb_${al}_$rep.json | grep value)"
done; done
