# batch geometry: 4-strip workgroups when every tile row fits the chip at once, vs forced 8
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/fit; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_shard.py tests/test_gpu_goldens.py tests/test_gpu_sparse_kernels.py tests/test_gpu_sparse_random.py -m gpu > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for cfg in "2 99000 100000" "4 49000 50000" "8 29000 31000" "16 18000 22000" "64 18000 22000"; do
  set -- $cfg
  CHK=""; if [ $1 = 8 ] || [ $1 = 16 ]; then CHK=--check; fi
  timeout -k 10 150 python tools/batch_bench.py --pairs $1 --lo $2 --hi $3 --tileBx 256 $CHK >> $O/auto.jsonl 2>>$O/err.log || { tail $O/err.log; exit 1; }
  GSA_KROW_NS=8 timeout -k 10 120 python tools/batch_bench.py --pairs $1 --lo $2 --hi $3 --tileBx 256 >> $O/ns8.jsonl 2>>$O/err.log || { tail $O/err.log; exit 1; }
done
python -c "
import json
for a,b in zip(open('$O/auto.jsonl'),open('$O/ns8.jsonl')):
    a,b=json.loads(a),json.loads(b); print(a['pairs'],a['lengths'],'auto',a['value'],a['seconds'],'ns8',b['value'],b['seconds'])
"
