#!/usr/bin/env python
"""Experiment: gemm_bl_kernel (B staged through LDS, shared by 4 row bands) against the
default gemm_kernel tiles (B read per wave from L2) and hipBLASLt on the train step's dense
shapes; GCG_GEMM_BL=1 selects the LDS-B tiles. Results must be bitwise equal (same k order)."""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from graphconvgeo_amd import dense  # noqa: E402
from graphconvgeo_amd.sparse import empty_dense  # noqa: E402
from tools.exp_xtg_blocks import time_op  # noqa: E402

PEAK = 157.3


def main():
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    cases = [("P.W2+b2 (fused shape, plain)", 840_000, 300, 930),
             ("dP = G.W2^T", 840_000, 930, 300),
             ("Z2 = h.W2", 1_400_000, 300, 930),
             ("dh = dZ2.W2^T", 1_400_000, 930, 300)]
    for name, M, K, N in cases:
        A = empty_dense(M, K, dev).copy_(torch.randn((M, K), generator=g, device=dev) * 0.1)
        W = torch.randn((K, N), generator=g, device=dev) * 0.05
        Wp = dense._WeightCache().get(W, False)
        out = empty_dense(M, N, dev)
        f = 2.0 * M * K * N
        os.environ.pop("GCG_GEMM_BL", None)
        ref = dense.gemm(A, Wp).clone()
        t0 = time_op(lambda: dense.gemm(A, Wp, out=out), 7)
        line = f"{name}: default {t0:.3f} ms ({f / t0 / 1e9:.1f} TF)"
        for v in ("1", "2"):
            os.environ["GCG_GEMM_BL"] = v
            o2 = dense.gemm(A, Wp)
            same = bool(torch.equal(o2, ref))
            t1 = time_op(lambda: dense.gemm(A, Wp, out=out), 7)
            line += f" | LDS-B{v} {t1:.3f} ms ({f / t1 / 1e9:.1f} TF, bitwise={same})"
            del o2
        os.environ.pop("GCG_GEMM_BL", None)
        tt = time_op(lambda: torch.matmul(A, W), 7)
        print(line + f" | hipBLASLt {tt:.3f} ms ({f / tt / 1e9:.1f} TF)", flush=True)
        del A, out, ref
    # fused output layer
    T, K, C = 840_000, 300, 930
    P = empty_dense(T, K, dev).copy_(torch.randn((T, K), generator=g, device=dev) * 0.1)
    W = torch.randn((K, C), generator=g, device=dev) * 0.05
    b = torch.randn(C, generator=g, device=dev) * 0.01
    y = torch.randint(0, C, (T,), generator=g, device=dev).to(torch.int32)
    Wp = dense._WeightCache().get(W, False)
    res = {}
    for bl in (0, 1, 2):
        if bl:
            os.environ["GCG_GEMM_BL"] = str(bl)
        G = empty_dense(T, C, dev)
        loss = torch.empty(T, device=dev)
        hits = torch.empty(T, device=dev)

        def run():
            dense._fused(P, Wp, b, y, 1.0 / T, None, G, loss, hits)
        run()
        res[bl] = (G.clone(), loss.clone(), hits.clone())
        ms = time_op(run, 7)
        print(f"fused {('LDS-B%d' % bl) if bl else 'default'}: {ms:.3f} ms "
              f"({2.0 * T * K * C / ms / 1e9:.1f} TF)", flush=True)
        os.environ.pop("GCG_GEMM_BL", None)
    for bl in (1, 2):
        print(f"fused LDS-B{bl} vs default: max |dG| "
              f"{float((res[bl][0] - res[0][0]).abs().max()):.3e}, max |dloss| "
              f"{float((res[bl][1] - res[0][1]).abs().max()):.3e}, hits equal "
              f"{bool(torch.equal(res[bl][2], res[0][2]))}")


if __name__ == "__main__":
    main()
