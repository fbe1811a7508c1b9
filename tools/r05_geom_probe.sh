#!/bin/bash
# Headline (configs[2], 100k sparse) under each K-rows single-pair geometry (GSA_KROW_NS / GSA_KROW_K):
# (4, 4) the default, (2, 4) and (4, 2) spread the pair over twice the workgroups, (2, 2) four times.
set -e
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$ROOT/gpurun_out/${1:-geom}; mkdir -p $O
for g in "4 4" "2 4" "4 2" "2 2" "4 4"; do
  set -- $g
  GSA_KROW_NS=$1 GSA_KROW_K=$2 timeout -k 10 120 python3 $ROOT/bench.py --steps 10 --warmup 2 --no-10k --no-config5 \
      --config4-pairs 0 --full-batch-pairs 0 --no-cpu-baseline > $O/ns$1_k$2.json 2> $O/ns$1_k$2.err
  python3 -c "import json,sys; d=json.load(open('$O/ns$1_k$2.json')); print('ns=$1 k=$2', d['value'], d['ms_per_step'], d['golden_match'])"
done
