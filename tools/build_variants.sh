#!/bin/bash
# Experiment builds of libgsa with extra defines: build_variants.sh name:"-DA=1 -DB=2" ...
# -> gpuseqalign_amd/libgsa_<name>.so (loaded only by tools/knob_probe.py via GSA_LIB).
set -e
cd "$(dirname "$0")/../gpuseqalign_amd/csrc"
mkdir -p build/var
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c nw_check.hip -o build/var/nw_check.o
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c nw_trace_dev.hip -o build/var/nw_trace_dev.o
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c nw_scan.hip -o build/var/nw_scan.o
hipcc -O3 -std=c++17 -fPIC -c nw_trace.cpp -o build/var/nw_trace.o
for spec in "$@"; do
  name="${spec%%:*}"; defs="${spec#*:}"
  for f in gsa_capi nw_strip nw_lane; do
    hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $defs -c -x hip $f.hip -o build/var/$f.$name.o &
  done
  wait
  hipcc --offload-arch=gfx950 -shared -fPIC build/var/gsa_capi.$name.o build/var/nw_strip.$name.o build/var/nw_lane.$name.o build/var/nw_trace.o build/var/nw_check.o build/var/nw_trace_dev.o build/var/nw_scan.o -o ../libgsa_$name.so
done
