#!/bin/bash
# diagnostic / A-B variants of libgsa.so: NAME "DEFINES" "SOURCES" -> gpuseqalign_amd/libgsa_NAME.so,
# the listed sources (csrc file names) rebuilt with DEFINES and linked with the default objects of
# the others (each source keeps its Makefile scheduler flags: K-rows translation units the
# iterative-ilp scheduler).  e.g. tools/r06_variant_build.sh kled -DGSA_KR_BLOCK_LEDGER=1 "nw_krow.hip nw_krowx.hip"
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
C=$ROOT/gpuseqalign_amd/csrc
make -s -C $C -j8
n=$1; defs=$2; srcs=$3
mkdir -p /tmp/vb_$n
objs_new=""
excl="^$"
for f in $srcs; do
  b=${f%.hip}
  sched=""
  case $b in nw_krow|nw_krowx|nw_lane|nw_strip) sched="-mllvm -amdgpu-sched-strategy=iterative-ilp";; esac
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $sched $defs -c $C/$f -o /tmp/vb_$n/$b.o &
  objs_new="$objs_new /tmp/vb_$n/$b.o"
  excl="$excl|/$b.o$"
done
wait
objs=$(ls $C/build/*.o | grep -Ev "$excl")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $ROOT/gpuseqalign_amd/libgsa_$n.so $objs $objs_new
echo built gpuseqalign_amd/libgsa_$n.so
