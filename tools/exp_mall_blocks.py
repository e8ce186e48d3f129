#!/usr/bin/env python
"""Column blocks sized for the Infinity Cache: World H.Z (K = 300) as ceil(300 / w) SpMMs over
separate w-column Z blocks (empty_dense layout: w = 32 -> one 128-B line per gathered row, a
1.4M x 32 block = 179 MB, inside the 256 MB MALL), against the one full-width launch. Each block
re-reads the (col, val) stream; every output column is the same storage-order sum (bitwise).
HIP events, mean of 10 launch sets after 3 warm-ups; both graphs."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphconvgeo_amd import sparse as gs  # noqa: E402
from graphconvgeo_amd.synth import CONFIGS, synthetic_graph  # noqa: E402

K = 300
dev = torch.device("cuda:0")
cfg = CONFIGS["twitter-world"]
kinds = (sys.argv[1] if len(sys.argv) > 1 else "uniform,powerlaw").split(",")


def timed(fn, reps=10):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


for kind in kinds:
    H = synthetic_graph(cfg.n_nodes, cfg.n_edges, kind=kind)
    n = H.shape[0]
    A = gs.DeviceCSR.from_scipy(H, dev, symmetric=True)
    for mode in dict.fromkeys([gs.resolve_auto(A), "rowwise", "ordered"]):
        Z = gs.empty_dense(n, K, dev).copy_(torch.randn((n, K), device=dev))
        Y = gs.empty_dense(n, K, dev)
        ref = gs.spmm(A, Z, mode=mode).clone()
        base = timed(lambda: gs.spmm(A, Z, out=Y, mode=mode))
        print(f"{kind} {mode} plain {base:.3f} ms", flush=True)
        for w in (32, 48, 64, 96):
            bounds = [(a, min(a + w, K)) for a in range(0, K, w)]
            zb = [gs.empty_dense(n, b - a, dev).copy_(Z[:, a:b]) for a, b in bounds]
            yb = [gs.empty_dense(n, b - a, dev) for a, b in bounds]
            ms = timed(lambda: [gs.spmm(A, z, out=y, mode=mode) for z, y in zip(zb, yb)])
            one = timed(lambda: gs.spmm(A, zb[0], out=yb[0], mode=mode))
            ok = all(torch.equal(y, ref[:, a:b]) for y, (a, b) in zip(yb, bounds))
            print(f"{kind} {mode} blocks w={w:3d} x{len(bounds)} {ms:.3f} ms (x{ms / base:.3f}; "
                  f"one block {one:.3f} ms) bitwise={ok}", flush=True)
            del zb, yb
        del Z, Y, ref
        torch.cuda.empty_cache()
    del A
