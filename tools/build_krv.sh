#!/bin/bash
# A/B builds of nw_krow.hip correct variants (GSA_KRV bits): gpuseqalign_amd/libgsa_krv<bits>.so
set -e
cd "$(dirname "$0")/../gpuseqalign_amd/csrc"
make -s
mkdir -p build/krv
for k in "$@"; do
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -DGSA_KRV=$k -c nw_krow.hip -o build/krv/nw_krow.$k.o &
done
wait
for k in "$@"; do
  hipcc -shared -fPIC --offload-arch=gfx950 -o ../libgsa_krv$k.so $(ls build/*.o | grep -v nw_krow.o) build/krv/nw_krow.$k.o
done
