#!/usr/bin/env python
"""The bench's headline launch alone (bench.spmm_variant: World graph, K = 300, empty_dense
operands, auto mode, default gather hint) on the power-law and the uniform graph, for A/Bs of
kernel builds (GCG_LIB names the library). HIP events, mean of 20 after 3 warm-ups, 3 rounds;
one JSON line per graph."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphconvgeo_amd import sparse as gs  # noqa: E402
from graphconvgeo_amd.synth import CONFIGS, synthetic_graph  # noqa: E402

dev = torch.device("cuda:0")
cfg = CONFIGS["twitter-world"]
K = 300
for kind in os.environ.get("KINDS", "powerlaw,uniform").split(","):
    H = synthetic_graph(cfg.n_nodes, cfg.n_edges, kind=kind)
    A = gs.DeviceCSR.from_scipy(H, dev, symmetric=True)
    g = torch.Generator(device=dev).manual_seed(0)
    Z = gs.empty_dense(H.shape[0], K, dev).copy_(torch.randn((H.shape[0], K), generator=g, device=dev))
    Y = gs.empty_dense(H.shape[0], K, dev)
    mode = gs.resolve_auto(A) if hasattr(gs, "resolve_auto") else "auto"
    f = lambda: gs.spmm(A, Z, out=Y, mode=mode)  # noqa: E731
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    res = []
    for _ in range(3):
        s.record()
        for _ in range(20):
            f()
        e.record()
        torch.cuda.synchronize()
        res.append(round(s.elapsed_time(e) / 20, 4))
    print(json.dumps({"graph": kind, "mode": mode, "ms": res, "lib": os.environ.get("GCG_LIB", "tree")}), flush=True)
    del A, Z, Y
