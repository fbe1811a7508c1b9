#!/bin/bash
# Timing-experiment build: the current tree with one source file patched by a python expression
# (knobs live here, not in the product sources).  usage:
#   tools/build_patch_variant.sh NAME FILE 'PY-EXPR on s'      e.g.
#   tools/build_patch_variant.sh noq nw_krow.hip 's.replace("qn[k][u] = lds_ld(", "qn[k][u] = qc[k][u] ^ 1 + 0*lds_ld(")'
#   tools/build_patch_variant.sh kst nw_krow.hip @tools/patches/krow_stamps.py   (a script that rewrites s)
# -> gpuseqalign_amd/libgsa_<NAME>.so (GSA_LIB=... for the timing tools).  Results may be WRONG.
set -e
NAME=$1; FILE=$2; EXPR=$3
ROOT=$(cd "$(dirname "$0")/.." && pwd)
D=$ROOT/build/patch_$NAME
rm -rf $D && mkdir -p $D/gpuseqalign_amd/csrc
(cd $ROOT/gpuseqalign_amd/csrc && tar --exclude=./build -cf - .) | (cd $D/gpuseqalign_amd/csrc && tar -xf -)
cp -r $ROOT/include $D/
(cd $ROOT && python3 - "$D/gpuseqalign_amd/csrc/$FILE" "$EXPR") <<'PY'
import sys
p, expr = sys.argv[1], sys.argv[2]
s = open(p).read()
if expr.startswith("@"):
    ns = {"s": s}
    exec(open(expr[1:]).read(), ns)
    t = ns["s"]
else:
    t = eval(expr, {"s": s})
assert t != s, "patch changed nothing"
open(p, "w").write(t)
PY
make -s -C $D/gpuseqalign_amd/csrc -j8 OUT=$ROOT/gpuseqalign_amd/libgsa_$NAME.so
