#!/usr/bin/env python
"""Experiment: cost of the SpMM epilogue variants (bias, rectify, rectify gate bytes and the
gate's row stride) on the layer-1 propagate H . Z1 (mlpconv.py:73-77). HIP events, mean of
reps, alternating variants so clock drift hits all of them alike."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphconvgeo_amd import sparse as gs  # noqa: E402
from graphconvgeo_amd.synth import CONFIGS, synthetic_graph  # noqa: E402

config = sys.argv[1] if len(sys.argv) > 1 else "twitter-us"
cfg = CONFIGS[config]
dev = torch.device("cuda:0")
H = synthetic_graph(cfg.n_nodes, cfg.n_edges)
A = gs.DeviceCSR.from_scipy(H, dev, symmetric=True)
n, K = H.shape[0], 300
Z = gs.empty_dense(n, K, dev).copy_(torch.randn((n, K), device=dev))
Y = gs.empty_dense(n, K, dev)
b = torch.randn(K, device=dev) * 0.1
gates = {ld: torch.empty((n, ld), dtype=torch.uint8, device=dev)[:, :K] for ld in (300, 320, 384)}
variants = {
    "plain": lambda: gs.spmm(A, Z, out=Y),
    "bias": lambda: gs.spmm(A, Z, bias=b, out=Y),
    "bias+relu": lambda: gs.spmm(A, Z, bias=b, act="relu", out=Y),
    "bias+relu+gate300": lambda: gs.spmm(A, Z, bias=b, act="relu", out=Y, gate=gates[300]),
    "bias+relu+gate320": lambda: gs.spmm(A, Z, bias=b, act="relu", out=Y, gate=gates[320]),
    "bias+relu+gate384": lambda: gs.spmm(A, Z, bias=b, act="relu", out=Y, gate=gates[384]),
}
for fn in variants.values():
    fn()
torch.cuda.synchronize()
times = {k: [] for k in variants}
for rnd in range(6):
    for name, fn in variants.items():
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(5)]
        for a, e in evs:
            a.record()
            fn()
            e.record()
        torch.cuda.synchronize()
        times[name] += [a.elapsed_time(e) for a, e in evs]
print(config, "mode", gs.resolve_auto(A))
for name, t in times.items():
    print(f"{name:22s} {np.mean(t):.4f} ms  (min {np.min(t):.4f})")
