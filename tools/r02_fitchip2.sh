# threshold probe: 4 vs 8 strips per workgroup for 12-64 pairs of 18-22k
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/fit2; mkdir -p $O
for n in 12 16 24 32 64; do
  for ns in 4 8; do
    GSA_KROW_NS=$ns timeout -k 10 120 python tools/batch_bench.py --pairs $n --tileBx 256 > $O/r.json 2>>$O/err.log || { tail $O/err.log; exit 1; }
    python -c "import json; d=json.load(open('$O/r.json')); print($n, $ns, d['value'], d['seconds'])" | tee -a $O/res.txt
  done
done
