#!/bin/bash
# Timing-experiment build: the current tree compiled with extra hipcc flags (compiler scheduling
# options).  usage: tools/build_flag_variant.sh NAME 'EXTRA FLAGS' -> gpuseqalign_amd/libgsa_<NAME>.so
set -e
NAME=$1; EXTRA=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
D=$ROOT/build/flag_$NAME
rm -rf $D && mkdir -p $D/gpuseqalign_amd/csrc
(cd $ROOT/gpuseqalign_amd/csrc && tar --exclude=./build -cf - .) | (cd $D/gpuseqalign_amd/csrc && tar -xf -)
cp -r $ROOT/include $D/
make -s -C $D/gpuseqalign_amd/csrc -j8 OUT=$ROOT/gpuseqalign_amd/libgsa_$NAME.so \
    HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-label $EXTRA"
