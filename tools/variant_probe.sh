#!/bin/bash
# Compare experiment builds of libgsa on one GPU box: variant_probe.sh OUTDIR name1 name2 ...
# (name "cur" = the in-tree libgsa.so, otherwise gpuseqalign_amd/libgsa_<name>.so).  Per variant:
# the full-fill parity ladder (tools/lane_quick.py) and the lane probe at 10k columns.
set -e
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$1
shift
mkdir -p $OUT
cd $ROOT
for v in "$@"; do
  if [ "$v" = cur ]; then lib=""; else lib=$ROOT/gpuseqalign_amd/libgsa_$v.so; fi
  echo "== $v" | tee -a $OUT/probe.txt
  GSA_LIB=$lib timeout -k 10 120 python tools/lane_quick.py > $OUT/quick_$v.txt 2>&1 || { tail -5 $OUT/quick_$v.txt; exit 1; }
  tail -1 $OUT/quick_$v.txt | tee -a $OUT/probe.txt
  GSA_LIB=$lib ROWS=${ROWS:-64,1024,10000} NSS=${NSS:-2} timeout -k 10 180 python tools/lane_probe.py 10000 2>/dev/null | tee -a $OUT/probe.txt || exit 1
done
