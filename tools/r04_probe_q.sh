#!/bin/bash
# Score int8 profile check + config 5 A/B, then the asm profile / halo / progress-read variants of the
# fill: golden parity under each, headline A/B, config 5 A/B of the asm profile reads.
set -e
L=$PWD/gpuseqalign_amd
bash tools/r04_ks_q8.sh
GSA_KROW_Q8=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_score.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/score_q16.log 2>&1 || { tail -20 gpurun_out/score_q16.log; exit 1; }
echo "score int16 profile: $(tail -1 gpurun_out/score_q16.log)"
for v in qasm pasm qp; do
  GSA_LIB=$L/libgsa_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_goldens.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gold_$v.log 2>&1 || { tail -20 gpurun_out/gold_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/gold_$v.log)"
done
GSA_LIB=$L/libgsa_qasm.so timeout -k 10 300 python -u -m pytest tests/test_gpu_score.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/score_qasm.log 2>&1 || { tail -20 gpurun_out/score_qasm.log; exit 1; }
echo "score qasm: $(tail -1 gpurun_out/score_qasm.log)"
bash tools/r04_ab_lib.sh $L/libgsa_qasm.so $L/libgsa_hpart.so $L/libgsa_pasm.so $L/libgsa_qp.so
bash tools/r04_ab5_lib.sh $L/libgsa_qasm.so
