#!/usr/bin/env python
"""Which bitwise mode should 'auto' pick on hub-free matrices? ordered (planned tasks) vs
rowwise (plan-less, one wave per row) -- and fast for reference -- on the products of the
training step, interleaved rounds in one process (CDNA rule 24): H.Z on the World uniform and
power-law graphs and the US graph, X.W1 (64-nnz rows, W1 cache-resident) at US and World.
Z in the library's empty_dense layout (ld 304). HIP events, mean of 10 after 3 warm-ups."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphconvgeo_amd import sparse as gs  # noqa: E402
from graphconvgeo_amd.synth import CONFIGS, synthetic_features, synthetic_graph  # noqa: E402

dev = torch.device("cuda:0")
K = 300


def timed(fn, reps=10):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return round(s.elapsed_time(e) / reps, 3)


cases = []
for cname, kind in (("twitter-world", "uniform"), ("twitter-world", "powerlaw"),
                    ("twitter-us", "powerlaw")):
    cfg = CONFIGS[cname]
    cases.append((f"{cname} {kind} H.Z", synthetic_graph(cfg.n_nodes, cfg.n_edges, kind=kind), True))
for cname in ("twitter-us", "twitter-world"):
    cfg = CONFIGS[cname]
    cases.append((f"{cname} X.W1", synthetic_features(cfg.n_nodes, cfg.n_features, nnz_per_row=64), False))
for what, M, sym in cases:
    A = gs.DeviceCSR.from_scipy(M, dev, symmetric=sym)
    Z = gs.empty_dense(M.shape[1], K, dev).copy_(torch.randn((M.shape[1], K), device=dev))
    Y = gs.empty_dense(M.shape[0], K, dev)
    res = {"auto_now": gs.resolve_auto(A), "max_row": int(A.max_row_nnz()),
           "mean_row": round(A.nnz / max(1, A.n_rows), 1)}
    ref = gs.spmm(A, Z, mode="ordered").clone()
    for rnd in range(3):
        for mode in ("ordered", "rowwise", "fast"):
            res.setdefault(mode, []).append(timed(lambda: gs.spmm(A, Z, out=Y, mode=mode)))
            if mode != "fast" and rnd == 0:
                assert torch.equal(Y, ref), f"{mode} not bitwise"
    print(json.dumps({"case": what, **res}), flush=True)
    del A, Z, Y, ref
    torch.cuda.empty_cache()
