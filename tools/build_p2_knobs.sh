#!/bin/bash
# Timing-experiment builds of libgsa with GSA_P2KNOB bits set in nw_pair2.hip (results are wrong
# by design): gpuseqalign_amd/libgsa_p2k<bits>.so, loaded with GSA_LIB=... by the timing tools.
set -e
cd "$(dirname "$0")/../gpuseqalign_amd/csrc"
make -s
mkdir -p build/p2k
for k in "$@"; do
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -DGSA_P2KNOB=$k -c nw_pair2.hip -o build/p2k/nw_pair2.$k.o &
done
wait
for k in "$@"; do
  objs=$(ls build/*.o | grep -v nw_pair2.o)
  hipcc -shared -fPIC --offload-arch=gfx950 -o ../libgsa_p2k$k.so $objs build/p2k/nw_pair2.$k.o
done
