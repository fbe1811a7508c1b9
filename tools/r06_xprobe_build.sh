#!/bin/bash
# diagnostic builds of the expansion linked with the default objects: each argument NAME=DEFINES
# (e.g. xp1="-DGSA_EXPAND_PROBE=1", xst1="-DGSA_EXPAND_STORE=1") -> gpuseqalign_amd/libgsa_NAME.so,
# nw_expand.hip and the fused kernel's translation unit (nw_krowx.hip) rebuilt with DEFINES.
# GSA_EXPAND_PROBE = 1: one add per cell, 2: no interior stores, 3: no pass-1 row / header-column
# loads (results wrong); GSA_EXPAND_STORE = 1: nontemporal stores, 2: write-through (sc1)
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
C=$ROOT/gpuseqalign_amd/csrc
make -s -C $C -j8
for spec in "$@"; do
  n=${spec%%=*}; defs=${spec#*=}
  mkdir -p /tmp/xb_$n
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $defs -c $C/nw_expand.hip -o /tmp/xb_$n/nw_expand.o &
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -mllvm -amdgpu-sched-strategy=iterative-ilp $defs -c $C/nw_krowx.hip -o /tmp/xb_$n/nw_krowx.o &
  wait
  objs=$(ls $C/build/*.o | grep -v "nw_expand.o\|nw_krowx.o")
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $ROOT/gpuseqalign_amd/libgsa_$n.so $objs /tmp/xb_$n/nw_expand.o /tmp/xb_$n/nw_krowx.o
done
