#!/usr/bin/env python
"""Profiling driver for rocprofv3 --pmc passes: 3 launches of the bench's SpMM (Twitter-World
H . Z, K = 300) on the power-law or the uniform graph in the given mode (default ordered)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphconvgeo_amd import sparse as gs  # noqa: E402
from graphconvgeo_amd.synth import CONFIGS, synthetic_graph  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "powerlaw"
mode = sys.argv[2] if len(sys.argv) > 2 else "ordered"
cfg = CONFIGS["twitter-world"]
dev = torch.device("cuda:0")
H = synthetic_graph(cfg.n_nodes, cfg.n_edges, kind=kind)
A = gs.DeviceCSR.from_scipy(H, dev, symmetric=True)
Z = gs.empty_dense(H.shape[0], 300, dev).copy_(torch.randn((H.shape[0], 300), device=dev))
Y = gs.empty_dense(H.shape[0], 300, dev)
gs.spmm(A, Z, out=Y, mode=mode)  # plan
torch.cuda.synchronize()
for _ in range(3):
    gs.spmm(A, Z, out=Y, mode=mode)
torch.cuda.synchronize()
print("done", kind, gs.resolve_auto(A) if mode == "auto" else mode)
