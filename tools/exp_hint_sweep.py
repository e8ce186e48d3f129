#!/usr/bin/env python
"""Gather-hint hot-set size re-swept after the non-temporal output stores (round 5): the bench's
headline launch (World power-law, K = 300, ordered, empty_dense operands) with
sparse.GATHER_HINT_HOT_BYTES in {16, 24, 32, 48, 64} MiB and GATHER_HINT_MIN_REUSE in {2, 4}
(and no hint), interleaved rounds in one process; HIP events, mean of 20. Bitwise the same
output in every setting (the hint is cache policy only)."""
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
H = synthetic_graph(cfg.n_nodes, cfg.n_edges)
g = torch.Generator(device=dev).manual_seed(0)
Z = gs.empty_dense(H.shape[0], K, dev).copy_(torch.randn((H.shape[0], K), generator=g, device=dev))
Y = gs.empty_dense(H.shape[0], K, dev)
settings = [(None, None)] + [(mb, r) for r in (4.0, 2.0) for mb in (16, 24, 32, 48, 64)]
res = {str(s): [] for s in settings}
ref = None
for rnd in range(3):
    for mb, reuse in settings:
        A = gs.DeviceCSR.from_scipy(H, dev, symmetric=True)  # fresh: the hint is cached per H
        gs.GATHER_HINT = mb is not None
        if mb is not None:
            gs.GATHER_HINT_HOT_BYTES = mb << 20
            gs.GATHER_HINT_MIN_REUSE = reuse
        f = lambda: gs.spmm(A, Z, out=Y, mode="ordered")  # noqa: E731
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        if ref is None:
            ref = Y.clone()
        elif rnd == 0:
            assert torch.equal(Y, ref), (mb, reuse)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(20):
            f()
        e.record()
        torch.cuda.synchronize()
        res[str((mb, reuse))].append(round(s.elapsed_time(e) / 20, 4))
        del A
print(json.dumps({"what": "hot-set MiB, min reuse -> ms (3 rounds)", **res}), flush=True)
