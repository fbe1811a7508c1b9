# A/B of variant libraries on one box: fused 100k full fill (pitched), alternating, 3 rounds
# usage: LIBS="name1 name2" [PAIR=10k REPS=20] bash tools/r06_ab.sh   (default = libgsa.so)
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/r06_ab.log
: > $L
for round in 1 2 3; do
  for lib in default $LIBS; do
    so=""; [ "$lib" != default ] && so=gpuseqalign_amd/libgsa_$lib.so
    GSA_LIB=$so timeout -k 10 120 python -u tools/r06_full100k.py --pitched --reps ${REPS:-4} --pair ${PAIR:-100k} --tag "$lib" >> $L 2>&1
  done
done
grep "^{" $L | python3 -c "
import sys, json, collections
d = collections.defaultdict(list)
for l in sys.stdin:
    j = json.loads(l); d[j['tag']].append((j['ms_mean'], j['ms_min'], j['align_cost']))
for k, v in d.items(): print(k, v)"
