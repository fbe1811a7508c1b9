#!/bin/bash
# Experiment build of the lane kernel + C ABI from a git revision: build_rev_variant.sh REV NAME
# -> gpuseqalign_amd/libgsa_<NAME>.so (the other objects from the normal in-tree build).
set -e
REV=${1:-HEAD}
NAME=${2:-head}
cd "$(dirname "$0")/../gpuseqalign_amd/csrc"
make -s -j8
mkdir -p build/rev_$NAME
git show $REV:gpuseqalign_amd/csrc/nw_lane.hip > build/rev_$NAME/nw_lane.hip
git show $REV:gpuseqalign_amd/csrc/gsa_capi.hip > build/rev_$NAME/gsa_capi.hip
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I. -c build/rev_$NAME/nw_lane.hip -o build/rev_$NAME/nw_lane.o &
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I. -I../../include -c build/rev_$NAME/gsa_capi.hip -o build/rev_$NAME/gsa_capi.o &
wait
hipcc --offload-arch=gfx950 -shared -fPIC build/nw_strip.o build/rev_$NAME/nw_lane.o build/nw_check.o build/nw_trace_dev.o \
  build/nw_scan.o build/rev_$NAME/gsa_capi.o build/nw_trace.o -o ../libgsa_$NAME.so
