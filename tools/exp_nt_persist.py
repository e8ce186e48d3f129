#!/usr/bin/env python
"""Persistent vs one-workgroup-per-tile NT GEMM (round 4, gcg_gemm_nt_f32, GCG_NT_PERSIST), on the
output layer's Twitter-World shapes, interleaved in one process: forward P.W2 + b2 (840k x 300 x
930), dP = G.W2^T (840k x 930 x 300), the reference order's h.W2 (1.4M x 300 x 930). HIP events,
mean of 10 after 5 warm-ups, TFLOP/s against the 157.3 TF f32 MFMA peak."""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphconvgeo_amd import dense  # noqa: E402
from graphconvgeo_amd.sparse import empty_dense  # noqa: E402

dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(5)


def timed(fn, reps=10):
    for _ in range(5):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


cases = []
for name, M, K, N, bias in (("P.W2+b2", 840_000, 300, 930, True), ("G.W2^T", 840_000, 930, 300, False),
                            ("h.W2", 1_400_000, 300, 930, False)):
    A = empty_dense(M, K, dev).copy_(torch.randn((M, K), generator=g, device=dev) * 0.1)
    W = (torch.rand((K, N), generator=g, device=dev) * 2 - 1) * math.sqrt(6.0 / (K + N))
    Bt = dense._WeightCache().get(W, True)
    b = torch.randn(N, generator=g, device=dev) if bias else None
    C = empty_dense(M, N, dev)
    cases.append((name, M, K, N, A, Bt, b, C))
for rnd in range(int(os.environ.get("ROUNDS", "3"))):
    for name, M, K, N, A, Bt, b, C in cases:
        for p in ("0", "1"):
            os.environ["GCG_NT_PERSIST"] = p
            ms = timed(lambda: dense.gemm_nt(A, Bt, bias=b, out=C))
            tf = 2.0 * M * K * N / (ms * 1e-3) / 1e12
            print(json.dumps({"round": rnd, "case": name, "persist": int(p), "ms": round(ms, 3),
                              "TFLOPs": round(tf, 1), "frac": round(tf / 157.3, 3)}), flush=True)
