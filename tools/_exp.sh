#!/bin/bash
# scratch experiment driver (one GPU call)
set -e
O=gpuseqalign_amd/../gpurun_out/$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for ns in 2 3 4; do
  GSA_LANE_NS=$ns timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench_ns$ns.json 2> $O/bench_ns$ns.err || { tail $O/bench_ns$ns.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_ns$ns.json'));print($ns, d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
  GSA_LANE_NS=$ns timeout -k 10 200 python tools/batch_bench.py --mode full --pairs 64 > $O/batch_ns$ns.json 2>/dev/null || exit 1
  tail -1 $O/batch_ns$ns.json
done
