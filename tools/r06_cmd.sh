set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/r06_s16.log
: > $L
for lib in "" pa pb; do
  so=""; [ -n "$lib" ] && so=gpuseqalign_amd/libgsa_$lib.so
  GSA_LIB=$so timeout -k 10 120 python -u tools/r06_stamps100k.py _$lib >> $L 2>&1
done
grep -v amdgpu.ids $L | grep "^{" | python3 -c "
import sys, json
for l in sys.stdin:
    j = json.loads(l)
    print('fused', j['ms'], j['cost_ok'], 'strip end first/last', j['strip_end_us']['first'], j['strip_end_us']['last'], j['tasks_done_per_500us'])"
