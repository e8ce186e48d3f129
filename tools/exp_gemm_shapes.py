#!/usr/bin/env python
"""Experiment: TFLOP/s of the MFMA GEMM (csrc/dense.hip) vs hipBLASLt across K and N at
M = 840k rows, to see how much per-workgroup prologue/epilogue costs (grows relative to the
K loop as K shrinks)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphconvgeo_amd import dense  # noqa: E402
from graphconvgeo_amd.sparse import empty_dense  # noqa: E402
from tools.bench_dense import time_op  # noqa: E402

dev = torch.device("cuda:0")
M = int(os.environ.get("M", "840000"))
for K, N in [(300, 930), (600, 930), (1200, 930), (300, 1024), (300, 512), (300, 256), (2400, 930)]:
    A = empty_dense(M, K, dev).normal_()
    W = torch.randn(K, N, device=dev) * 0.05
    Wp = dense._WeightCache().get(W, False)
    out = empty_dense(M, N, dev)
    f = 2.0 * M * K * N
    ms = time_op(lambda: dense.gemm(A, Wp, out=out), 5)
    tm = time_op(lambda: torch.matmul(A, W), 5)
    print(f"K={K:5d} N={N:5d}  ours {ms:7.3f} ms {f/ms/1e9:6.1f} TF   torch {tm:7.3f} ms {f/tm/1e9:6.1f} TF",
          flush=True)
    del A, W, Wp, out
