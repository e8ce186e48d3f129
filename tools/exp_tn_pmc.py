#!/usr/bin/env python
"""Profiling driver: 3 launches of the split-K weight-gradient GEMM (gcg_gemm_tn_f32) at the
World dW2 shape 840k x 300 x 930 (for rocprofv3 --pmc passes, tools/gpu/pmc_nt.sh DRIVER=)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphconvgeo_amd import dense  # noqa: E402
from graphconvgeo_amd.sparse import empty_dense  # noqa: E402

dev = torch.device("cuda:0")
A = empty_dense(840_000, 300, dev).normal_(0, 0.1)
B = empty_dense(840_000, 930, dev).normal_(0, 0.1)
for _ in range(3):
    dense.gemm_tn(A, B)
torch.cuda.synchronize()
print("done")
