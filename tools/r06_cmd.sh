set -e
bash tools/r06_prof.sh r06prof4
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u bench.py > gpurun_out/r06_bench_final2.json 2> gpurun_out/r06_bench_final2.err
python3 -c "
import json
j = json.loads(open('gpurun_out/r06_bench_final2.json').read().strip().splitlines()[-1])
print(j['value'], j['ms_per_step'], j['roofline']['kernel_ms'], j['roofline']['frac'])
print('100k full', (j.get('fill_100k_full') or {}).get('kernel_ms'), (j.get('fill_100k_full') or {}).get('hbm_frac'))
print('batch', (j.get('full_batch') or {}).get('hbm_frac'))
"
