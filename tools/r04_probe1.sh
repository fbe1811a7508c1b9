#!/bin/bash
# round-4 probe: (1) the K-rows sparse fill of the configs[1] size (10k) in its geometries,
# (2) the full batch (pitched, paired) at 2, 4 and 8 lane strips per workgroup.
set -e
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$ROOT/gpurun_out/${1:-r04_probe1}; mkdir -p $O
cd $ROOT
for kn in "4 4" "2 4" "4 2" "2 2"; do
  set -- $kn
  GSA_KROW_K=$1 GSA_KROW_NS=$2 timeout -k 10 120 python -u tools/gpu_perf.py --shapes "" --sizes 10000,20000 > $O/sparse_k$1_ns$2.jsonl 2>&1
  echo "K=$1 NS=$2"; grep sparse $O/sparse_k$1_ns$2.jsonl | cut -c1-120
done
for ns in 4 8 2; do
  GSA_LANE_NS=$ns timeout -k 10 200 python -u tools/full_ab.py --rounds 1 > $O/full_ns$ns.jsonl 2>&1
  echo "lane NS=$ns"; grep leg $O/full_ns$ns.jsonl
done
