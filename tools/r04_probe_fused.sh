# fused 10k probe: XR pass 1 in its plain (PT 2) and fused (PT 3, GSA_XR_PT3) instances, tiles skipped:
# knob 1 as is, 65 without the per-boundary publication (results wrong)
set -e
mkdir -p gpurun_out
for v in "0 1" "1 1" "1 65" "0 1" "1 65" "1 1"; do set -- $v; echo "pt3 $1 knob $2"; GSA_XR_PT3=$1 GSA_EXPAND_KNOB=$2 timeout -k 10 100 python -u tools/full_ab.py --batch 0 --rounds 1 2>/dev/null | grep '"fused": false'; done > gpurun_out/r04_f9.log 2>&1
cat gpurun_out/r04_f9.log
