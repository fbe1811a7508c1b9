#!/bin/bash
# whole-bench A/B of library builds (LIBS="cur name ..."; libgsa_<name>.so), no CPU legs
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
O=gpurun_out/${1:-bench_ab}; mkdir -p $O
for rep in $(seq ${REPS:-2}); do
  for lib in ${LIBS:-cur}; do
    L=$PWD/gpuseqalign_amd/libgsa.so; [ $lib != cur ] && L=$PWD/gpuseqalign_amd/libgsa_$lib.so
    GSA_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 2 > $O/b_${lib}_$rep.json 2> $O/b_${lib}_$rep.err || { tail $O/b_${lib}_$rep.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/b_${lib}_$rep.json').read().strip().splitlines()[-1])
c5=d.get('config5',{}).get('modes',{})
print('$lib', $rep, 'head', d['ms_per_step'], '10k', d['fill_10k_full']['value'], 'c4', d['config4']['value'], 'fb', d['full_batch']['value'], 'sw', c5.get('SW-LG',{}).get('kernel_ms'), 'ag', c5.get('NW-AG',{}).get('kernel_ms'))"
  done
done
