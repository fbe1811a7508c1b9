set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/r06_s17.log
: > $L
timeout -k 10 120 python -u tools/r06_stamps100k.py _st >> $L 2>&1
grep -v amdgpu.ids $L | grep "^{" | python3 -c "
import sys, json
for l in sys.stdin:
    j = json.loads(l)
    print('fused', j['ms'], j['cost_ok'], 'strip end first/last', j['strip_end_us']['first'], j['strip_end_us']['last'], j['tasks_done_per_500us'])"
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_full100k.py tests/test_gpu_parity.py > gpurun_out/r06_t17.log 2>&1 || { tail -30 gpurun_out/r06_t17.log; exit 1; }
tail -3 gpurun_out/r06_t17.log
