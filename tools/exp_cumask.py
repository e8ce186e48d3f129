#!/usr/bin/env python
"""Experiment: CU-partitioned overlap. The gather SpMM runs on a stream masked to a subset of
the CUs (hipExtStreamCreateWithCUMask) and the MFMA weight gradient on a stream masked to the
complement. Is the SpMM still HBM-bound on fewer CUs, and does the pair then overlap?"""
from __future__ import annotations

import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from graphconvgeo_amd import dense, sparse as gs  # noqa: E402
from graphconvgeo_amd.synth import CONFIGS, synthetic_graph  # noqa: E402
from tools.exp_xtg_blocks import time_op  # noqa: E402

_hip = C.CDLL("libamdhip64.so")


def masked_stream(dev, keep):
    n = torch.cuda.get_device_properties(dev).multi_processor_count
    words = [0] * ((n + 31) // 32)
    cnt = 0
    for i in range(n):
        if keep(i):
            words[i // 32] |= 1 << (i % 32)
            cnt += 1
    arr = (C.c_uint32 * len(words))(*words)
    h = C.c_void_p()
    rc = _hip.hipExtStreamCreateWithCUMask(C.byref(h), C.c_uint32(len(words)), arr)
    assert rc == 0, rc
    return torch.cuda.ExternalStream(h.value, device=dev), cnt


def main():
    cfg = CONFIGS["twitter-world"]
    dev = torch.device("cuda:0")
    H = synthetic_graph(cfg.n_nodes, cfg.n_edges)
    Hd = gs.DeviceCSR.from_scipy(H, dev, symmetric=True)
    K, Cc, T = 300, 930, 840_000
    Z = gs.empty_dense(cfg.n_nodes, K, dev)
    Z.copy_(torch.randn(cfg.n_nodes, K, device=dev))
    Y = gs.spmm(Hd, Z)
    P = gs.empty_dense(T, K, dev)
    P.copy_(torch.randn(T, K, device=dev))
    G = gs.empty_dense(T, Cc, dev)
    G.copy_(torch.randn(T, Cc, device=dev))
    W = dense.gemm_tn(P, G)
    main_s = torch.cuda.current_stream(dev)

    def on(stream, fn):
        def run():
            stream.wait_stream(main_s)
            with torch.cuda.stream(stream):
                fn()
            main_s.wait_stream(stream)
        return run

    def spmm():
        gs.spmm(Hd, Z, out=Y)

    def tn():
        dense.gemm_tn(P, G, out=W)

    print("all CUs: spmm", round(time_op(spmm, 5), 3), "gemm_tn", round(time_op(tn, 5), 3),
          flush=True)
    for mod in (8, 4, 2):
        a, na = masked_stream(dev, lambda i: i % mod != mod - 1)
        b, nb = masked_stream(dev, lambda i: i % mod == mod - 1)
        t_a = time_op(on(a, spmm), 5)
        t_b = time_op(on(b, tn), 5)

        def both(k):
            def run():
                a.wait_stream(main_s)
                b.wait_stream(main_s)
                with torch.cuda.stream(b):
                    tn()
                with torch.cuda.stream(a):
                    for _ in range(k):
                        spmm()
                main_s.wait_stream(a)
                main_s.wait_stream(b)
            return run
        print(f"spmm on {na} CUs {t_a:.3f} | gemm_tn on {nb} CUs {t_b:.3f} | "
              f"both {time_op(both(1), 5):.3f} | tn + 3 spmm {time_op(both(3), 5):.3f}",
              flush=True)
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
