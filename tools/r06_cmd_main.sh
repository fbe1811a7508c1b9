# fused 100k stamps, the full-fill GPU tests, and a short bench (fill fields only)
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-s}
L=gpurun_out/r06_$T.log
: > $L
timeout -k 10 120 python -u tools/r06_stamps100k.py _$T >> $L 2>&1
grep -v amdgpu.ids $L | grep "^{" | python3 -c "
import sys, json
for l in sys.stdin:
    j = json.loads(l)
    print('fused', j['ms'], j['cost_ok'], 'strip end first/last', j['strip_end_us']['first'], j['strip_end_us']['last'], j['task_dur_us'], j['tasks_done_per_500us'])"
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_full100k.py tests/test_gpu_parity.py > gpurun_out/r06_t$T.log 2>&1 || { tail -30 gpurun_out/r06_t$T.log; exit 1; }
tail -2 gpurun_out/r06_t$T.log
timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline --config4-pairs 0 --no-config5 > gpurun_out/r06_b$T.json 2> gpurun_out/r06_b$T.err
python3 -c "
import json
j = json.loads(open('gpurun_out/r06_b$T.json').read().strip().splitlines()[-1])
print('headline', j['value'], j['roofline']['kernel_ms'])
f = j['fill_10k_full']; print('10k', f['kernel_ms'], f['hbm_frac'], f['align_cost'])
f = j['fill_100k_full']; print('100k', f['kernel_ms'], f['hbm_write_GBps'], f['hbm_frac'], f['align_cost'], f['golden_align_cost'])
f = j['full_batch']; print('batch', f['seconds'], f['hbm_write_GBps'], f['hbm_frac'], f['pairs_matching_golden'], f['passes'].get('pass1_ms'), f['passes'].get('pass2_ms'), f['first_launch_ms'])
"
