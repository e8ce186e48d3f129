#!/usr/bin/env python
"""Profiling driver: 3 launches each of the fused output kernel (default tile), the plain
register-B MFMA GEMM, the NT GEMM (forward 840k x 300 x 930, input gradient 840k x 930 x 300)
and the split-K weight gradient at Twitter-World's output-layer shapes (for rocprofv3 --pmc
passes)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphconvgeo_amd import dense  # noqa: E402
from graphconvgeo_amd.sparse import empty_dense  # noqa: E402

dev = torch.device("cuda:0")
T, K, C = 840_000, 300, 930
P = empty_dense(T, K, dev).normal_(0, 0.1)
W = torch.randn(K, C, device=dev) * 0.05
Wp = dense._WeightCache().get(W, False)
b = torch.zeros(C, device=dev)
y = torch.randint(0, C, (T,), device=dev, dtype=torch.int32)
G = empty_dense(T, C, dev)
loss = torch.empty(T, device=dev)
hits = torch.empty(T, device=dev)
for _ in range(3):
    dense._fused(P, Wp, b, y, 1.0 / T, None, G, loss, hits)
for _ in range(3):
    dense.gemm(P, Wp, bias=b, out=G)
Wt = dense._WeightCache().get(W, True)
for _ in range(3):
    dense.gemm_nt(P, Wt, bias=b, out=G)
dP = empty_dense(T, K, dev)
for _ in range(3):
    dense.gemm_nt(G, Wp, out=dP)
for _ in range(3):  # the weight gradient dW2 = P^T . G (bf16x6 split-K, dense.TN_MATH)
    dense.gemm_tn(P, G)
torch.cuda.synchronize()
print("done")
