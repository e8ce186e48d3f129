#!/usr/bin/env python
"""Fused output layer (P.W2 + b2 -> softmax-CE, mlpconv.py:88-95) tile variants after the
buffer-descriptor B loads, interleaved rounds on one device, outputs compared bitwise with the
default: 8-wave workgroups (2 row bands share every B address through L1; GCG_GEMM_8W=1 one B
register set, =2 the 8-part split ring), and RT = 4 at 1 workgroup per CU (GCG_GEMM_OCC2=0)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphconvgeo_amd import dense  # noqa: E402
from graphconvgeo_amd.sparse import empty_dense  # noqa: E402

variants = {"default": {}, "8w-split8": {"GCG_GEMM_8W": "2"}, "8w": {"GCG_GEMM_8W": "1"},
            "rt4-1wg": {"GCG_GEMM_OCC2": "0"}}
knobs = {k for v in variants.values() for k in v}
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
        for name, env in variants.items():
            for k in knobs:
                os.environ.pop(k, None)
            os.environ.update(env)
            f()
            torch.cuda.synchronize()
            if rnd == 0:
                outs[name] = (G.clone(), loss.clone(), hits.clone())
            s.record()
            for _ in range(10):
                f()
            e.record()
            torch.cuda.synchronize()
            res.setdefault(name, []).append(round(2.0 * T * K * C / (s.elapsed_time(e) / 10) / 1e9, 1))
    for k in knobs:
        os.environ.pop(k, None)
    bitwise = {n: all(torch.equal(a, c) for a, c in zip(outs["default"], o)) for n, o in outs.items()}
    print(json.dumps({"shape": f"{T}x{K}x{C}", "TFLOPs": res, "bitwise_vs_default": bitwise}), flush=True)
    del P, G, outs
    torch.cuda.empty_cache()
