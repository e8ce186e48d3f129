#!/usr/bin/env python
"""Profiling driver: 3 launches each of the bf16x6 NT GEMM with the pre-split weight
(gcg_gemm_nt math bf16x6; tile via argv[1], default 0) on the output-layer shapes: forward
840k x 300 x 930 (+ b2) and input gradient 840k x 930 x 300 (for rocprofv3 --pmc passes)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphconvgeo_amd import dense  # noqa: E402
from graphconvgeo_amd.sparse import empty_dense  # noqa: E402

tile = int(sys.argv[1]) if len(sys.argv) > 1 else 0
dev = torch.device("cuda:0")
T, K, C = 840_000, 300, 930
P = empty_dense(T, K, dev).normal_(0, 0.1)
W = torch.randn(K, C, device=dev) * 0.05
b = torch.zeros(C, device=dev)
Wt = dense._WeightCache().get(W, True)
Wp = dense._WeightCache().get(W, False)
G = empty_dense(T, C, dev)
for _ in range(3):
    dense.gemm_nt(P, Wt, bias=b, out=G, math="bf16x6", tile=tile)
dP = empty_dense(T, K, dev)
for _ in range(3):
    dense.gemm_nt(G, Wp, out=dP, math="bf16x6", tile=tile)
torch.cuda.synchronize()
print("done")
