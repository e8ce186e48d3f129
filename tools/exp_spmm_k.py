#!/usr/bin/env python
"""Headline SpMM H.Z across the dense width K on the World graphs: the reference's hidden sizes
(tensormain.py: default 500, tuning 64..1568 and 512..2304, 1500) besides the configs' 300.
Z/Y in the library's layout (empty_dense), the mode 'auto' resolves to, HIP events (mean of 10
after 3 warm-ups), edge-centric GB/s and its fraction of 8 TB/s."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphconvgeo_amd import sparse as gs  # noqa: E402
from graphconvgeo_amd.synth import CONFIGS, synthetic_graph  # noqa: E402

dev = torch.device("cuda:0")
cfg = CONFIGS["twitter-world"]
Ks = [int(k) for k in os.environ.get("KS", "64,128,256,300,500,512,800,1024,1500,2048").split(",")]
for kind in (sys.argv[1] if len(sys.argv) > 1 else "powerlaw,uniform").split(","):
    H = synthetic_graph(cfg.n_nodes, cfg.n_edges, kind=kind)
    A = gs.DeviceCSR.from_scipy(H, dev, symmetric=True)
    n, nnz = H.shape[0], H.nnz
    mode = gs.resolve_auto(A)
    for K in Ks:
        Z = gs.empty_dense(n, K, dev).copy_(torch.randn((n, K), device=dev))
        Y = gs.empty_dense(n, K, dev)
        for _ in range(3):
            gs.spmm(A, Z, out=Y, mode=mode)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(10):
            gs.spmm(A, Z, out=Y, mode=mode)
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / 10
        B = 4 * (n + 1) + 8 * nnz + 4 * K * nnz + 4 * K * n
        print(json.dumps({"graph": kind, "mode": mode, "K": K, "ld": Z.stride(0), "ms": round(ms, 3),
                          "GBps": round(B / ms / 1e6, 1), "frac": round(B / ms / 1e6 / 8000, 3)}),
              flush=True)
        del Z, Y
        torch.cuda.empty_cache()
    del A
