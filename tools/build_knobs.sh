#!/bin/bash
# Timing-experiment builds of libgsa with GSA_KNOB bits set (results are wrong by design).
set -e
cd "$(dirname "$0")/../gpuseqalign_amd/csrc"
mkdir -p build/knob
for k in "$@"; do
  for f in gsa_capi nw_strip; do
    hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -DGSA_KNOB=$k -c -x hip $f.hip -o build/knob/$f.$k.o &
  done
  wait
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c nw_check.hip -o build/knob/nw_check.o
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c nw_trace_dev.hip -o build/knob/nw_trace_dev.o
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c nw_scan.hip -o build/knob/nw_scan.o
  hipcc -O3 -std=c++17 -fPIC -c nw_trace.cpp -o build/knob/nw_trace.o
  hipcc --offload-arch=gfx950 -shared -fPIC build/knob/gsa_capi.$k.o build/knob/nw_strip.$k.o build/knob/nw_trace.o build/knob/nw_check.o build/knob/nw_trace_dev.o build/knob/nw_scan.o -o ../libgsa_k$k.so
done
