# output-buffer placement probe under the expansion's task orders (GSA_EXPAND_RR): 1 round-robin
# over pairs (default), 2 the same with each pair rotated, 3 shuffled
mkdir -p gpurun_out/obuf
for rr in 1 2 3; do
  GSA_EXPAND_RR=$rr timeout -k 10 300 python -u tools/r05_outbuf_probe.py > gpurun_out/obuf/f_rr$rr.txt 2>> gpurun_out/obuf/f.err || exit 1
done
