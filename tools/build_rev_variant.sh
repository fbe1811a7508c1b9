#!/bin/bash
# A/B build of the whole library from a git revision: build_rev_variant.sh REV NAME
# -> gpuseqalign_amd/libgsa_<NAME>.so (loaded by the timing tools with GSA_LIB=...).
set -e
REV=${1:-HEAD}
NAME=${2:-head}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
D=$ROOT/gpuseqalign_amd/csrc/build/rev_$NAME
rm -rf $D && mkdir -p $D
git -C $ROOT archive $REV gpuseqalign_amd/csrc include | tar -x -C $D
make -s -C $D/gpuseqalign_amd/csrc -j8 OUT=$ROOT/gpuseqalign_amd/libgsa_$NAME.so
