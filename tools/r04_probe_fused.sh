# fused 10k probe: XR pass 1 with the fused instance's stores/publication (GSA_XR_PT3) vs plain
set -e
mkdir -p gpurun_out
for v in 0 1; do echo "pt3 $v"; GSA_XR_PT3=$v GSA_EXPAND_KNOB=1 timeout -k 10 100 python -u tools/full_ab.py --batch 0 --rounds 1 2>/dev/null; done > gpurun_out/r04_f5.log 2>&1
cat gpurun_out/r04_f5.log
