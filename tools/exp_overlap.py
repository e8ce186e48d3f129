#!/usr/bin/env python
"""Experiment: does an MFMA-bound kernel (the split-K weight gradient P^T . G) overlap an
HBM-bound CSR gather (H . Z) when the two are launched on different streams? Twitter-World
shapes; HIP events around (a) each alone, (b) both on one stream, (c) both on two streams."""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from graphconvgeo_amd import dense, sparse as gs  # noqa: E402
from graphconvgeo_amd.synth import CONFIGS, synthetic_graph  # noqa: E402
from tools.exp_xtg_blocks import time_op  # noqa: E402


def main():
    cfg = CONFIGS["twitter-world"]
    dev = torch.device("cuda:0")
    H = synthetic_graph(cfg.n_nodes, cfg.n_edges)
    Hd = gs.DeviceCSR.from_scipy(H, dev, symmetric=True)
    K, C, T = 300, 930, 840_000
    Z = gs.empty_dense(cfg.n_nodes, K, dev)
    Z.copy_(torch.randn(cfg.n_nodes, K, device=dev))
    Y = gs.spmm(Hd, Z)
    P = gs.empty_dense(T, K, dev)
    P.copy_(torch.randn(T, K, device=dev))
    G = gs.empty_dense(T, C, dev)
    G.copy_(torch.randn(T, C, device=dev))
    W = dense.gemm_tn(P, G)
    side = torch.cuda.Stream(dev)
    main_s = torch.cuda.current_stream(dev)

    def spmm():
        gs.spmm(Hd, Z, out=Y)

    def tn():
        dense.gemm_tn(P, G, out=W)

    def serial():
        spmm()
        tn()

    def concurrent():
        side.wait_stream(main_s)
        with torch.cuda.stream(side):
            tn()
        spmm()
        main_s.wait_stream(side)

    def concurrent_x3():  # a gather chain with one weight gradient beside it
        side.wait_stream(main_s)
        with torch.cuda.stream(side):
            tn()
        spmm()
        spmm()
        main_s.wait_stream(side)

    res = {}
    for name, fn in (("spmm", spmm), ("gemm_tn", tn), ("serial", serial),
                     ("concurrent", concurrent), ("spmm_x2", lambda: (spmm(), spmm())),
                     ("concurrent_spmm_x2", concurrent_x3)):
        res[name] = round(time_op(fn, 7), 3)
        print(name, res[name], flush=True)
    print(res)


if __name__ == "__main__":
    main()
