set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/r06_stage.log
: > $L
GSA_LIB=gpuseqalign_amd/libgsa_noex.so timeout -k 10 120 python -u tools/r06_stamps100k.py _noex2 >> $L 2>&1 || true
timeout -k 10 120 python -u tools/r06_stamps100k.py _s25 >> $L 2>&1
python3 -c "
import numpy as np
for tag in ['noex2','s25']:
    d=np.load(f'gpurun_out/r06_stamps100k_{tag}.npz'); st=d['st'].astype(np.int64); n=int(d['nstrips'])
    s=st[:4*n].reshape(n,4)
    t0=s[:,0].min(); end=(s[:,1]-t0)/100.
    clk=(s[:,3]-s[:,2])/((s[:,1]-s[:,0])*10.)
    e=end.reshape(-1,4)
    print(tag,'first end',round(end[0],1),'last',round(end.max(),1),'clk first',round(clk[0],3),'cyc/step first',round((s[0,3]-s[0,2])/100000,1),'ticket lag',round(float(np.median(np.diff(e[:,0]))),2))
"
grep "^{" $L | cut -c1-400
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_full100k.py tests/test_gpu_parity.py > gpurun_out/r06_ts25.log 2>&1 || { tail -30 gpurun_out/r06_ts25.log; exit 1; }
tail -2 gpurun_out/r06_ts25.log
