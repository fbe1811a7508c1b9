#!/bin/bash
# Experiment builds of the lane kernel only: build_lane_variants.sh name:"-DA=1" ...
# -> gpuseqalign_amd/libgsa_<name>.so (the other objects from the normal in-tree build).
set -e
cd "$(dirname "$0")/../gpuseqalign_amd/csrc"
make -s -j8
mkdir -p build/var
for spec in "$@"; do
  name="${spec%%:*}"; defs="${spec#*:}"
  ( hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $defs -c nw_lane.hip -o build/var/nw_lane.$name.o &&
    hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $defs -c gsa_capi.hip -o build/var/gsa_capi.$name.o &&
    hipcc --offload-arch=gfx950 -shared -fPIC build/nw_strip.o build/var/nw_lane.$name.o build/nw_check.o build/nw_trace_dev.o build/nw_scan.o build/var/gsa_capi.$name.o build/nw_trace.o -o ../libgsa_$name.so ) &
done
wait
