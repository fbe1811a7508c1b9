set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/r06_hl_ab3.log
: > $L
for round in 1 2 3; do
  for lib in default p2w2 p2w3; do
    so=""; [ "$lib" != default ] && so=gpuseqalign_amd/libgsa_$lib.so
    r=$(GSA_LIB=$so timeout -k 10 120 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --config4-pairs 0 --no-10k --no-100k-full --no-rank-share --full-batch-pairs 0 --no-config5 2>/dev/null | grep '^{' | python3 -c "import sys,json; j=json.loads(sys.stdin.read()); print(j['ms_per_step'], j['roofline']['kernel_ms'])")
    echo "$lib $r" >> $L
  done
done
cat $L
