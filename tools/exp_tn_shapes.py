#!/usr/bin/env python
"""Experiment: split-K TN GEMM (gcg_gemm_tn_f32) tile variants (GCG_TN="MG,NG,PD") on the
train step's weight-gradient shapes: dW2 = P^T.G (propagate-first), h^T.dZ2 (reference order)
and the dense-head W1 gradient X_head^T.G (both orientations)."""
from __future__ import annotations

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from graphconvgeo_amd import dense  # noqa: E402
from graphconvgeo_amd.sparse import empty_dense  # noqa: E402
from tools.exp_xtg_blocks import time_op  # noqa: E402

SHAPES = [(840_000, 300, 930), (1_400_000, 300, 930), (1_400_000, 164, 300),
          (1_400_000, 192, 300), (1_400_000, 256, 300), (1_400_000, 300, 192),
          (1_400_000, 300, 256)]
VARIANTS = ["1,2,8", "1,1,8", "1,2,4", "1,1,16", "1,2,12"]


def main():
    dev = torch.device("cuda:0")
    for R, M, N in SHAPES:
        A = empty_dense(R, M, dev).copy_(torch.randn(R, M, device=dev))
        B = empty_dense(R, N, dev).copy_(torch.randn(R, N, device=dev))
        ref = dense.gemm_tn(A, B)
        line = []
        for v in VARIANTS:
            os.environ["GCG_TN"] = v
            out = dense.gemm_tn(A, B)
            ok = bool(torch.allclose(out, ref, rtol=1e-4, atol=1e-2))
            ms = time_op(lambda: dense.gemm_tn(A, B, out=out), 5)
            line.append(f"{v}: {ms:.3f} ms {2 * R * M * N / ms / 1e9:.1f} TF{'' if ok else ' MISMATCH'}")
        os.environ.pop("GCG_TN")
        print((R, M, N), " | ".join(line), flush=True)
        del A, B


if __name__ == "__main__":
    main()
