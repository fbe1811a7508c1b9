set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/r06_s22.log
: > $L
timeout -k 10 120 python -u tools/r06_stamps100k.py _s22 >> $L 2>&1
grep "^{" $L
