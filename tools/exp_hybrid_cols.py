#!/usr/bin/env python
"""Experiment: X^T . G (the W1 gradient, grad of mlpconv.py:71) with the dense-head split
(sparse.HYBRID_MAX_COLS most frequent columns at density >= HYBRID_MIN_DENSITY on the split-K
MFMA GEMM, side stream; the rest a CSR gather): time per head size, HIP events."""
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
G = gs.empty_dense(cfg.n_nodes, 300, dev).copy_(torch.randn(cfg.n_nodes, 300, device=dev))
counts = np.sort(np.bincount(X.indices, minlength=X.shape[1]))[::-1]
res = {}
for cols, dens in ((256, 0.02), (384, 0.005), (512, 0.005), (768, 0.002), (1024, 0.002)):
    gs.HYBRID_MAX_COLS, gs.HYBRID_MIN_DENSITY = cols, dens
    A = gs.DeviceCSR.from_scipy(X, dev)
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
    fh = A._dense_split[1].shape[1]
    res[f"{cols}/{dens}"] = {"head_cols": int(fh), "head_nnz_frac": round(float(counts[:fh].sum() / X.nnz), 3),
                             "ms": round(float(np.mean(ts)), 3)}
    del A
print(config, res)
