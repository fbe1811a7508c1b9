set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/r06_s10.log
: > $L
GSA_EXPAND_KNOB=1 GSA_FULL_FUSED=0 timeout -k 10 120 python -u tools/r06_full100k.py --reps 3 --pitched --timing --tag "knob1" >> $L 2>&1
GSA_FULL_FUSED=0 timeout -k 10 120 python -u tools/r06_full100k.py --reps 3 --pitched --timing --tag "base" >> $L 2>&1
timeout -k 10 120 python -u tools/r06_stamps100k.py _phase >> $L 2>&1
GSA_FULL_SPLIT=0 GSA_EXPAND_RR=1 timeout -k 10 200 python -u tools/batch_bench.py --mode full --pairs 64 --repeats 3 --warmup 1 >> $L 2>&1
grep -v amdgpu.ids $L | grep "^{" | python3 -c "
import sys, json
for l in sys.stdin:
    j = json.loads(l)
    if 'strip_end_us' in j: print('fused', j['ms'], j['cost_ok'], 'strip end first/last', j['strip_end_us']['first'], j['strip_end_us']['last'], j['tasks_done_per_500us'])
    elif 'tag' in j: print(j['tag'], j['ms_mean'], j['timing']['pass1_ms'], j['timing']['pass2_ms'], j['align_cost'])
    else: print('batch', j['value'], j.get('seconds'))"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_full100k.py tests/test_gpu_parity.py -k "not pipelined" > gpurun_out/r06_t10.log 2>&1 || true
tail -3 gpurun_out/r06_t10.log
