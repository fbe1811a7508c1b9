#!/bin/bash
# lane fill with / without the separate feeder wave: full-fill parity, then the 10k config-2
# pair and the 64-pair batch (the batch keeps 6 waves by default)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
O=gpurun_out/lane_feed; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_shard.py tests/test_gpu_check.py > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
GSA_LANE_FEED=1 GSA_LANE_NS=4 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "full or plain or lane" > $O/pytest_fd.txt 2>&1 || { tail -30 $O/pytest_fd.txt; exit 1; }
tail -2 $O/pytest_fd.txt
for rep in 1 2 3; do
  for fd in 0 1; do
    GSA_LANE_FEED=$fd timeout -k 10 120 python tools/batch_bench.py --mode full --pairs 1 --lo 10000 --hi 10000 --repeats 10 > $O/b1_${fd}_$rep.json 2>&1 || { tail $O/b1_${fd}_$rep.json; exit 1; }
    echo "feed=$fd rep=$rep 10k: $(grep -o '"value": [0-9.]*' $O/b1_${fd}_$rep.json)"
  done
done
