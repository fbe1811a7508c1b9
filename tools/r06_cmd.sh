set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/r06_px3.log
: > $L
for lib in g64 g64p11; do
  GSA_LIB=gpuseqalign_amd/libgsa_$lib.so GSA_FULL_FUSED=0 timeout -k 10 120 python -u tools/r06_full100k.py --pitched --timing --reps 2 --tag "$lib" >> $L 2>&1
done
grep "^{" $L | python3 -c "
import sys, json
for l in sys.stdin:
    j = json.loads(l)
    t = j.get('timing') or {}
    print(j['tag'], 'p2', t.get('pass2_ms'), 'GB/s/CU', round(j['bytes']/ (t.get('pass2_ms', 1e9)*1e-3)/1e9/64, 2))"
