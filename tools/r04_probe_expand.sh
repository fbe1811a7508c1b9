# pass-2 (expansion) geometry probe on the 64 x 20k full batch, same process: one workgroup per task
# (default) vs persistent workgroups (GSA_EXPAND_GRID) of 8 / 12 / 16 waves (GSA_EXPAND_WAVES), and
# both passes fused into one launch (GSA_FULL_FUSED=2) with GSA_FUSED_P1 pass-1 workgroups
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/full_ab.py --no-10k --rounds 1 --batch 64 --variants \
  "GSA_EXPAND_GRID=0" "GSA_EXPAND_WAVES=8" "GSA_EXPAND_GRID=0" "GSA_EXPAND_WAVES=8" "GSA_EXPAND_GRID=512,GSA_EXPAND_WAVES=8" "GSA_EXPAND_WAVES=8,GSA_EXPAND_MT=2" "GSA_EXPAND_GRID=0" "GSA_EXPAND_WAVES=8" > gpurun_out/r04_x2.log 2>&1
cat gpurun_out/r04_x2.log
