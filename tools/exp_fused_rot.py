#!/usr/bin/env python
"""Fused output layer (P.W2 + b2 -> softmax-CE, mlpconv.py:88-95) with the waves rotated over
the column slots per workgroup (GCG_GEMM_ROT=1) vs the fixed slot order: N = 930 fills 15 of the
16 64-column groups of a 4 x 256 row tile, so without rotation the short slot's wave may always
land on the same SIMD. Interleaved rounds on one device; outputs compared bitwise."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphconvgeo_amd import dense  # noqa: E402
from graphconvgeo_amd.sparse import empty_dense  # noqa: E402

dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
for T, K, C in ((840_000, 300, 930), (270_000, 300, 256)):
    P = empty_dense(T, K, dev).copy_(torch.randn((T, K), generator=g, device=dev) * 0.1)
    W = (torch.rand((K, C), generator=g, device=dev) * 2 - 1) * float(np.sqrt(6 / (K + C)))
    b = torch.randn(C, generator=g, device=dev) * 0.01
    y = torch.randint(0, C, (T,), generator=g, device=dev, dtype=torch.int32)
    Wp = dense._WeightCache().get(W, False)
    G = empty_dense(T, C, dev)
    loss = torch.empty(T, device=dev)
    hits = torch.empty(T, device=dev)
    f = lambda: dense._fused(P, Wp, b, y, 1.0 / T, None, G, loss, hits)  # noqa: E731
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    res, outs = {}, {}
    for rnd in range(3):
        for rot in ("0", "1"):
            os.environ["GCG_GEMM_ROT"] = rot
            f()
            torch.cuda.synchronize()
            if rnd == 0:
                outs[rot] = (G.clone(), loss.clone(), hits.clone())
            s.record()
            for _ in range(10):
                f()
            e.record()
            torch.cuda.synchronize()
            res.setdefault(rot, []).append(round(2.0 * T * K * C / (s.elapsed_time(e) / 10) / 1e9, 1))
    os.environ.pop("GCG_GEMM_ROT", None)
    bitwise = all(torch.equal(a, b) for a, b in zip(outs["0"], outs["1"]))
    print(json.dumps({"shape": f"{T}x{K}x{C}", "TFLOPs": res, "bitwise": bitwise}), flush=True)
    del P, G
    torch.cuda.empty_cache()
