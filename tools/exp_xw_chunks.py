#!/usr/bin/env python
"""X.W1 (mlpconv.py:71) split by columns of W1: does a narrower slice of the cache-resident W1
(60 MB at Twitter-World, 12 MB at Twitter-US: L2 / Infinity-Cache bound gathers) gather
faster? Full launch vs n column chunks, each its own launch (bitwise the same output: every
element keeps its storage-order sum). HIP events, mean of 10 after 3 warm-ups."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphconvgeo_amd import sparse as gs  # noqa: E402
from graphconvgeo_amd.synth import CONFIGS, synthetic_features  # noqa: E402

dev = torch.device("cuda:0")
K = 300


def timed(f, reps=10):
    for _ in range(3):
        f()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        f()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def bounds(n):
    step = (K + 4 * n - 1) // (4 * n) * 4
    return [(c, min(K, c + step)) for c in range(0, K, step)]


for name in sys.argv[1:] or ["twitter-us", "twitter-world"]:
    cfg = CONFIGS[name]
    X = synthetic_features(cfg.n_nodes, cfg.n_features)
    A = gs.DeviceCSR.from_scipy(X, dev)
    mode = gs.resolve_auto(A)
    W = gs.empty_dense(X.shape[1], K, dev).copy_(torch.randn((X.shape[1], K), device=dev))
    Y = gs.empty_dense(X.shape[0], K, dev)
    Yc = gs.empty_dense(X.shape[0], K, dev)
    ms = timed(lambda: gs.spmm(A, W, out=Y, mode=mode))
    print(json.dumps({"config": name, "nnz_X": X.nnz, "F": X.shape[1], "mode": mode,
                      "chunks": 1, "ms": round(ms, 3),
                      "gather_TBps": round(X.nnz * K * 4 / ms / 1e9, 2)}), flush=True)
    for n in (2, 3, 4, 8):
        bs = bounds(n)

        def run():
            for c0, c1 in bs:
                gs.spmm(A, W[:, c0:c1], out=Yc[:, c0:c1], mode=mode)
        msn = timed(run)
        print(json.dumps({"config": name, "chunks": n, "widths": [c1 - c0 for c0, c1 in bs],
                          "ms": round(msn, 3), "bitwise": bool(torch.equal(Y, Yc))}), flush=True)
    del A, W, Y, Yc
    torch.cuda.empty_cache()
