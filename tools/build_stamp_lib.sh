#!/bin/bash
# Diagnostic build: libgsa_p2stamp.so = libgsa with block stamps in the sparse single-pair kernels
# (GSA_KRSTAMP in nw_krow.hip) and the stamp export of gsa_capi.
set -e
cd "$(dirname "$0")/../gpuseqalign_amd/csrc"
make -s
mkdir -p build/p2k
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -DGSA_STAMP=1 -c gsa_capi.hip -o build/p2k/gsa_capi.stamp.o &
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -DGSA_KRSTAMP=1 -c nw_krow.hip -o build/p2k/nw_krow.stamp.o &
wait
hipcc -shared -fPIC --offload-arch=gfx950 -o ../libgsa_p2stamp.so $(ls build/*.o | grep -v "nw_krow.o\|gsa_capi.o") build/p2k/gsa_capi.stamp.o build/p2k/nw_krow.stamp.o
