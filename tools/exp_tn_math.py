#!/usr/bin/env python
"""gcg_gemm_tn f32 vs bf16x6 (gemm_tn6_partial_kernel) at the training step's shapes: World dW2
(P^T . G, 840k x 300 x 930; the propagate-first step's 531k distinct targets), the X-head
gradient (G^T . Xh as 1.4M x 256 x 300) and Twitter-US dW2 (270k x 300 x 256). HIP events,
mean of 10 after 3 warm-ups, alternated `--rounds` times; error vs float64 on sampled columns."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphconvgeo_amd import dense  # noqa: E402
from graphconvgeo_amd.sparse import empty_dense  # noqa: E402

ROUNDS = int(sys.argv[sys.argv.index("--rounds") + 1]) if "--rounds" in sys.argv else 2
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
for name, R, M, N in (("world dW2", 840_000, 300, 930), ("world dW2 distinct", 531_000, 300, 930),
                      ("world X head", 1_400_000, 256, 300), ("us dW2", 270_000, 300, 256)):
    A = empty_dense(R, M, dev).copy_(torch.randn((R, M), generator=g, device=dev) * 0.1)
    B = empty_dense(R, N, dev).copy_(torch.randn((R, N), generator=g, device=dev) * 0.01)
    cols = torch.randint(0, N, (8,), generator=g, device=dev)
    C64 = (A.double().T @ B[:, cols].double()).cpu().numpy()
    for _ in range(ROUNDS):
        for math in ("f32", "bf16x6"):
            f = lambda: dense.gemm_tn(A, B, math=math)  # noqa: E731
            for _ in range(3):
                C = f()
            torch.cuda.synchronize()
            err = float(np.abs(C[:, cols].double().cpu().numpy() - C64).max())
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(10):
                f()
            e.record()
            torch.cuda.synchronize()
            ms = s.elapsed_time(e) / 10
            print(json.dumps({"shape": name, "R": R, "M": M, "N": N, "math": math, "ms": round(ms, 4),
                              "TFLOPs": round(2.0 * R * M * N / (ms * 1e-3) / 1e12, 1),
                              "max_abs_err": err}), flush=True)
    del A, B
