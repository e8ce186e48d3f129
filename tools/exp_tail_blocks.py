#!/usr/bin/env python
"""Experiment: X^T . G (the W1 gradient, grad of mlpconv.py:71) with the CSR tail gather cut
into row blocks of X of TAIL_BLOCK_BYTES of G each (sparse.DeviceCSR.tmatmul), HIP events."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphconvgeo_amd import sparse as gs  # noqa: E402
from graphconvgeo_amd.synth import CONFIGS, synthetic_features  # noqa: E402

config = sys.argv[1] if len(sys.argv) > 1 else "twitter-us"
cfg = CONFIGS[config]
dev = torch.device("cuda:0")
X = synthetic_features(cfg.n_nodes, cfg.n_features, nnz_per_row=64)
A = gs.DeviceCSR.from_scipy(X, dev)
G = gs.empty_dense(cfg.n_nodes, 300, dev).copy_(torch.randn(cfg.n_nodes, 300, device=dev))
res = {}
for mb in (0, 256, 128, 64, 32):
    gs.TAIL_BLOCK_BYTES = mb << 20
    A.tmatmul(G, mode="fast")
    torch.cuda.synchronize()
    ts = []
    for _ in range(10):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        A.tmatmul(G, mode="fast")
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    res[mb] = round(float(np.mean(ts)), 3)
print(config, "ms by TAIL_BLOCK_MB (0 = one block):", res)
