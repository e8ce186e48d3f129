#!/usr/bin/env python
"""Per-op timings of the sparse products on the GCN path (HIP events, one MI355X).

  H.Z   (K = 300)            S.dot(H, .) layer 1                mlpconv.py:73
  H.Z2  (C = 930)            S.dot(H, .) layer 2, reference order mlpconv.py:90
  X.W1  (K = 300)            S.dot(X, W1)                       mlpconv.py:71   (W1 cache-resident)
  X^T.G (K = 300)            grad of S.dot(X, W1) w.r.t. W1

Bytes: the edge-centric model 4(N+1) + 8 nnz + 4 K nnz + 4 K N_out (every gathered row counted),
and for X.W1 also the compulsory model 4(N+1) + 8 nnz + 4 F K + 4 N K (W1 read once).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from graphconvgeo_amd import sparse as gs  # noqa: E402
from graphconvgeo_amd.synth import CONFIGS, synthetic_features, synthetic_graph  # noqa: E402


def edge_bytes(n_out, nnz, K):
    return 4 * (n_out + 1) + 8 * nnz + 4 * K * nnz + 4 * K * n_out


def time_op(fn, reps):
    fn()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in evs:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return float(np.mean([a.elapsed_time(b) for a, b in evs]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="twitter-world", choices=sorted(CONFIGS))
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--mode", default="auto")
    args = ap.parse_args()
    cfg = CONFIGS[args.config]
    dev = torch.device("cuda:0")
    H = synthetic_graph(cfg.n_nodes, cfg.n_edges)
    X = synthetic_features(cfg.n_nodes, cfg.n_features, nnz_per_row=64)
    A = gs.DeviceCSR.from_scipy(H, dev, symmetric=True)
    Xd = gs.DeviceCSR.from_scipy(X, dev)
    Xt = Xd.transpose()
    N, K, C, F = cfg.n_nodes, cfg.hidden, cfg.n_classes, cfg.n_features
    g = torch.Generator(device=dev).manual_seed(1)
    Z = torch.randn((N, K), generator=g, device=dev)
    Z2 = torch.randn((N, C), generator=g, device=dev)
    W1 = torch.randn((F, K), generator=g, device=dev)
    G = torch.randn((N, K), generator=g, device=dev)
    out = {}
    for name, fn, b_edge, extra in [
        ("H.Z", lambda: gs.spmm(A, Z, mode=args.mode), edge_bytes(N, H.nnz, K), {}),
        ("H.Z2", lambda: gs.spmm(A, Z2, mode=args.mode), edge_bytes(N, H.nnz, C), {}),
        ("X.W1", lambda: gs.spmm(Xd, W1, mode=args.mode), edge_bytes(N, X.nnz, K),
         {"compulsory_bytes": 4 * (N + 1) + 8 * X.nnz + 4 * F * K + 4 * N * K}),
        ("X^T.G", lambda: gs.spmm(Xt, G, mode=args.mode), edge_bytes(F, X.nnz, K),
         {"max_row_nnz": Xt.max_row_nnz()}),
    ]:
        ms = time_op(fn, args.reps)
        rec = {"ms": round(ms, 4), "edge_GBps": round(b_edge / (ms * 1e-3) / 1e9, 1)}
        for k, v in extra.items():
            rec[k] = v
            if k == "compulsory_bytes":
                rec["compulsory_GBps"] = round(v / (ms * 1e-3) / 1e9, 1)
        out[name] = rec
    print(json.dumps({"config": cfg.name, "nnz_H": H.nnz, "nnz_X": X.nnz, "mode": args.mode, "ops": out}))


if __name__ == "__main__":
    main()
