#!/bin/bash
# Timing-experiment builds of libgsa with GSA_KRKNOB bits set in nw_krow.hip (results are wrong
# by design): gpuseqalign_amd/libgsa_krk<bits>.so, loaded with GSA_LIB=... by the timing tools.
set -e
cd "$(dirname "$0")/../gpuseqalign_amd/csrc"
make -s
mkdir -p build/krk
for k in "$@"; do
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -DGSA_KRKNOB=$k -c nw_krow.hip -o build/krk/nw_krow.$k.o &
done
wait
for k in "$@"; do
  hipcc -shared -fPIC --offload-arch=gfx950 -o ../libgsa_krk$k.so $(ls build/*.o | grep -v nw_krow.o) build/krk/nw_krow.$k.o
done
