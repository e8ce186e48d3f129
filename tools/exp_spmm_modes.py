#!/usr/bin/env python
"""SpMM mode / task-size sweep on the Twitter-World graphs, K = 300: ordered vs fast vs
rowwise, task_nnz in {256, 512, 1024, 2048}. HIP events, mean of 10 after 3 warm-ups."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphconvgeo_amd import sparse as gs  # noqa: E402
from graphconvgeo_amd.synth import CONFIGS, synthetic_graph  # noqa: E402

kinds = (sys.argv[1] if len(sys.argv) > 1 else "powerlaw,uniform").split(",")
cfg = CONFIGS["twitter-world"]
dev = torch.device("cuda:0")
for kind in kinds:
    H = synthetic_graph(cfg.n_nodes, cfg.n_edges, kind=kind)
    A = gs.DeviceCSR.from_scipy(H, dev, symmetric=True)
    Z = torch.randn((H.shape[0], 300), device=dev)
    Y = gs.empty_dense(H.shape[0], 300, dev)
    sweep = os.environ.get("SWEEP", "ordered:0,ordered:256,ordered:1024,ordered:2048,fast:0,"
                                    "fast:256,fast:1024,fast:2048,rowwise:0,ordered:0")
    for mode, tn in [(m, int(t)) for m, t in (x.split(":") for x in sweep.split(","))]:
        for _ in range(3):
            gs.spmm(A, Z, out=Y, mode=mode, task_nnz=tn)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(10):
            gs.spmm(A, Z, out=Y, mode=mode, task_nnz=tn)
        e.record()
        torch.cuda.synchronize()
        print(f"{kind} {mode} task_nnz={tn} ms={s.elapsed_time(e) / 10:.3f}", flush=True)
    del A, Z, Y
