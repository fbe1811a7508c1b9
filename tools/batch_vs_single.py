"""Diagnostic: one pair through the single-pair entry point and through batched launches of
1 and 2 copies; prints header mismatches against the oracle for each."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import gpuseqalign_amd as gsa
import oracle
from tests._data import Golden, random_pair
G = Golden()
R, C = int(sys.argv[1]), int(sys.argv[2])
Y, X = random_pair(R, C, 5)
hr, hc, _, _, cost = oracle.sparse_headers(Y, X, G.blosum62, -11, gsa.sparse_tile_by(), 64)
dev = torch.device("cuda:0")
ts = torch.from_numpy(G.blosum62).to(dev)
tY, tX = torch.from_numpy(Y).to(dev), torch.from_numpy(X).to(dev)
g = gsa.sparse_geometry(R + 1, C + 1, 64)
with gsa.Engine(0) as e:
    try:
        r = e.align_sparse(Y, X, G.blosum62, -11, tileBx=64)
        print("single: hrow diff", int((r.hrow != hr).sum()), "hcol diff", int((r.hcol != hc).sum()), flush=True)
    except Exception as ex:
        print("single: error", ex, flush=True)
    for n in ((1, 2) if hasattr(e, "fill_batch_dev") and os.environ.get("GSA_LIB", "").find("v3") < 0 else ()):
        outs = [(torch.zeros(g.hrowElems, dtype=torch.int32, device=dev), torch.zeros(g.hcolElems, dtype=torch.int32, device=dev)) for _ in range(n)]
        try:
            e.fill_batch_dev([(tY.data_ptr(), R + 1, tX.data_ptr(), C + 1, (o[0].data_ptr(), o[1].data_ptr())) for o in outs],
                             ts.data_ptr(), 25, -11, mode="sparse", tileBx=64)
            e.sync()
            for k, o in enumerate(outs):
                print("batch", n, k, "hrow diff", int((o[0].cpu().numpy() != hr).sum()), "hcol diff", int((o[1].cpu().numpy() != hc).sum()), flush=True)
        except Exception as ex:
            print("batch", n, "error", ex, flush=True)
