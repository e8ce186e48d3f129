#!/usr/bin/env python
"""The Twitter-US training step's K = 300 SpMMs alone (X.W1, H.Z1 with bias + rectify + gate,
H.g1), for A/Bs of kernel builds: GCG_LIB names the library (graphconvgeo_amd._native). HIP
events, mean of 20 after 5 warm-ups; one JSON line."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphconvgeo_amd import sparse as gs  # noqa: E402
from graphconvgeo_amd.synth import CONFIGS, synthetic_features, synthetic_graph  # noqa: E402

dev = torch.device("cuda:0")
cfg = CONFIGS["twitter-us"]
K = cfg.hidden
H = synthetic_graph(cfg.n_nodes, cfg.n_edges)
X = synthetic_features(cfg.n_nodes, cfg.n_features, nnz_per_row=64)
A = gs.DeviceCSR.from_scipy(H, dev, symmetric=True)
Xd = gs.DeviceCSR.from_scipy(X, dev)
g = torch.Generator(device=dev).manual_seed(5)
W1 = gs.empty_dense(cfg.n_features, K, dev).normal_(generator=g)
Z1 = gs.empty_dense(cfg.n_nodes, K, dev).normal_(generator=g)
b1 = torch.randn(K, device=dev, generator=g)
gate = gs.empty_gate(cfg.n_nodes, K, dev)


def timed(fn, reps=20):
    for _ in range(5):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return round(s.elapsed_time(e) / reps, 4)


rec = {"lib": os.environ.get("GCG_LIB", "in-tree").rsplit("/", 1)[-1],
       "X.W1": timed(lambda: gs.spmm(Xd, W1)),
       "X.W1 mode": gs.resolve_auto(Xd),
       "H.Z1 relu gate": timed(lambda: gs.spmm(A, Z1, bias=b1, act="relu", gate=gate)),
       "H.g1": timed(lambda: gs.spmm(A, Z1)),
       "H mode": gs.resolve_auto(A)}
print(json.dumps(rec), flush=True)
