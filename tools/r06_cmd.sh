set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06_smoke.log 2>&1
tail -1 gpurun_out/r06_smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/r06_bench_final.json 2> gpurun_out/r06_bench_final.err
python3 -c "
import json
j = json.loads(open('gpurun_out/r06_bench_final.json').read().strip().splitlines()[-1])
print(j['value'], j['ms_per_step'], j['roofline']['kernel_ms'], j['roofline']['frac'])
f = j.get('fill_100k_full') or {}
print('100k full', f.get('kernel_ms'), f.get('hbm_frac'), f.get('align_cost'))
b = j.get('full_batch') or {}
print('batch', b.get('value'), b.get('hbm_frac'))
"
