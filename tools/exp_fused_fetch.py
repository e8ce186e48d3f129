#!/usr/bin/env python
"""Profiling driver for where the fused output layer's HBM reads come from (VERDICT r05 item 4:
FETCH_SIZE above the A operand): 3 launches of the fused layer (default tile, bf16x6) at
Twitter-World's shape (840k x 300 x 930) and 3 at the same rows with 64 classes, whose weight
planes (38 KB) cannot miss L2 -- so its fetch is A (and labels) alone, on this access pattern.
Run under `rocprofv3 --pmc FETCH_SIZE` and `--pmc TCC_HIT_sum TCC_MISS_sum` (tools/gpu/r06_fetch.sh)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphconvgeo_amd import dense  # noqa: E402
from graphconvgeo_amd.sparse import empty_dense  # noqa: E402

dev = torch.device("cuda:0")
T, K = 840_000, 300
P = empty_dense(T, K, dev).normal_(0, 0.1)
for C in (930, 64):
    W = torch.randn(K, C, device=dev) * 0.05
    Wp = dense._WeightCache().get(W, False)
    b = torch.zeros(C, device=dev)
    y = torch.randint(0, C, (T,), device=dev, dtype=torch.int32)
    G = empty_dense(T, C, dev)
    loss = torch.empty(T, device=dev)
    hits = torch.empty(T, device=dev)
    for _ in range(3):
        dense._fused(P, Wp, b, y, 1.0 / T, None, G, loss, hits)
    torch.cuda.synchronize()
    del G
print("done")
