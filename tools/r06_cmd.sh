set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/r06_px2.log
: > $L
for lib in "" xp1 xp6 xp7; do
  so=""; [ -n "$lib" ] && so=gpuseqalign_amd/libgsa_$lib.so
  for g in 64 256; do
    GSA_LIB=$so GSA_FULL_FUSED=0 GSA_EXPAND_GRID=$g timeout -k 10 120 python -u tools/r06_full100k.py --pitched --timing --reps 2 --tag "$lib g$g" >> $L 2>&1
  done
done
grep "^{" $L | python3 -c "
import sys, json
for l in sys.stdin:
    j = json.loads(l)
    t = j.get('timing') or {}
    print(j['tag'], j['ms_mean'], j['align_cost'], 'p1', t.get('pass1_ms'), 'p2', t.get('pass2_ms'), 'p2 GB/s', round(j['bytes']/ (t.get('pass2_ms', 1e9)*1e-3)/1e9, 1), 'clk', t.get('pass2_clock_ghz', t.get('clock')))"
