"""Diagnose the grouped two-pass full batch (GSA_FULL_GROUPS): per pair, which rows / columns differ
from the oracle, with and without a device sync before the call."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gpuseqalign_amd as gsa  # noqa: E402
import oracle  # noqa: E402
from tests._data import Golden, random_pair  # noqa: E402

os.environ["GSA_FULL_KERNEL"] = "twopass"
os.environ["GSA_KROW_NS"] = "4"
os.environ["GSA_FULL_FUSED"] = "0"
g = Golden()
sub = g.subst_data.matrix("blosum45")
pairs = [random_pair(r, c, 7 * r + c, alphabet=25) for r, c in ((2100, 900), (1, 5), (700, 2500), (64, 64), (4097, 300))]
dev = torch.device("cuda:0")
eng = gsa.Engine(0)
s = torch.from_numpy(np.ascontiguousarray(sub, dtype=np.int32)).to(dev)
ins = [(torch.from_numpy(Y).to(dev), torch.from_numpy(X).to(dev)) for Y, X in pairs]
lds = [gsa.full_pitch(len(X)) for _, X in pairs]
for groups in ["1", "3", "2", "5"]:
    for presync in (True, False):
        os.environ["GSA_FULL_GROUPS"] = groups
        bufs = [torch.full((len(Y) * ld + 64,), -7, dtype=torch.int32, device=dev) for (Y, _), ld in zip(pairs, lds)]
        if presync:
            torch.cuda.synchronize()
        eng.fill_batch_dev([(y.data_ptr(), len(y), x.data_ptr(), len(x), b.data_ptr() + 4 * 31)
                            for (y, x), b in zip(ins, bufs)], s.data_ptr(), 25, -5, mode="full", lds=lds)
        eng.sync()
        torch.cuda.synchronize()
        res = []
        for (Y, X), b, ld in zip(pairs, bufs, lds):
            M = b.cpu().numpy()[31:31 + len(Y) * ld].reshape(len(Y), ld)[:, :len(X)]
            S, _ = oracle.fill_full(Y, X, sub, -5)
            bad = M != S
            if not bad.any():
                res.append("ok")
            else:
                rr = np.where(bad.any(1))[0]
                cc = np.where(bad.any(0))[0]
                res.append(f"bad rows {rr.min()}..{rr.max()} ({len(rr)}) cols {cc.min()}..{cc.max()} ({len(cc)}) "
                           f"minus7 {(M == -7).sum()} of {M.size}")
        print("groups", groups, "presync", presync, res, flush=True)
