# output-buffer placement probe: the expansion's task order tuned per buffer (default) and fixed (1, 2)
mkdir -p gpurun_out/obuf
for rr in tuned 1 2; do
  if [ $rr = tuned ]; then unset GSA_EXPAND_RR; else export GSA_EXPAND_RR=$rr; fi
  timeout -k 10 300 python -u tools/r05_outbuf_probe.py > gpurun_out/obuf/g_$rr.txt 2>> gpurun_out/obuf/g.err || exit 1
done
