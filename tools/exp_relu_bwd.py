#!/usr/bin/env python
"""Rectify backward with the gate bytes + bias column sums (gcg_relu_backward_gate_f32) at the
training step's shapes: HIP events, mean of 20 after 3 warm-ups, effective GB/s over the bytes
it must move (read g and gate, write g)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphconvgeo_amd import sparse as gs  # noqa: E402

dev = torch.device("cuda:0")
for M, K in ((1_400_000, 300), (450_000, 300), (840_000, 930), (530_956, 930)):
    g = gs.empty_dense(M, K, dev).normal_()
    gate = gs.empty_gate(M, K, dev)
    gate.copy_(torch.randint(0, 3, (M, K), device=dev, dtype=torch.uint8))
    out = gs.empty_dense(M, K, dev)
    f = lambda: gs.relu_backward(g, gate=gate, out=out)  # noqa: E731
    for _ in range(3):
        f()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(20):
        f()
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / 20
    nbytes = M * K * (4 + 1 + 4)
    print(f"M={M} K={K} ms={ms:.3f} GB/s={nbytes / ms / 1e6:.0f}", flush=True)
    del g, gate, out
