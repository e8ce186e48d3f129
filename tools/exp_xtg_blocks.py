#!/usr/bin/env python
"""Experiment: dW1 = X^T . G (grad of S.dot(X, W1), mlpconv.py:71) with X^T split into column
blocks (= row blocks of X) so each pass gathers from a G block that fits the 256 MiB Infinity
Cache, partials summed. Compares against the single X^T SpMM. Twitter-World shapes."""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from graphconvgeo_amd import sparse as gs  # noqa: E402
from graphconvgeo_amd.synth import CONFIGS, synthetic_features  # noqa: E402


def time_op(fn, reps):
    fn()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(reps)]
    for a, b in evs:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in evs]))


def row_block(X: gs.DeviceCSR, r0: int, r1: int) -> gs.DeviceCSR:
    s, e = int(X.indptr[r0]), int(X.indptr[r1])
    return gs.DeviceCSR(X.indptr[r0:r1 + 1] - s, X.indices[s:e], X.data[s:e], (r1 - r0, X.n_cols),
                        validate=False)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="twitter-world")
    ap.add_argument("--blocks", default="2,4,8,16,32")
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    cfg = CONFIGS[args.config]
    dev = torch.device("cuda:0")
    X = synthetic_features(cfg.n_nodes, cfg.n_features, nnz_per_row=64)
    Xd = gs.DeviceCSR.from_scipy(X, dev)
    N, F, K = cfg.n_nodes, cfg.n_features, cfg.hidden
    G = gs.empty_dense(N, K, dev)
    G.copy_(torch.randn((N, K), device=dev))
    Xt = Xd.transpose()
    bytes_edge = 4 * (F + 1) + 8 * X.nnz + 4 * K * X.nnz + 4 * K * F
    res = {}
    ref = gs.spmm(Xt, G)
    ms = time_op(lambda: gs.spmm(Xt, G, out=ref), args.reps)
    res["single"] = {"ms": round(ms, 3), "edge_GBps": round(bytes_edge / ms / 1e6, 1)}
    print(res, flush=True)
    for nb in [int(x) for x in args.blocks.split(",")]:
        bounds = np.linspace(0, N, nb + 1).astype(int)
        blocks = [(int(a), int(b), row_block(Xd, int(a), int(b)).transpose())
                  for a, b in zip(bounds[:-1], bounds[1:])]
        parts = torch.empty((nb, F, (K + 3) // 4 * 4), device=dev)[:, :, :K]

        def run():
            for i, (a, b, T) in enumerate(blocks):
                gs.spmm(T, G[a:b], out=parts[i])
            return parts.sum(dim=0)

        out = run()
        err = float((out - ref).abs().max())
        ms = time_op(run, args.reps)

        def spmm_only():
            for i, (a, b, T) in enumerate(blocks):
                gs.spmm(T, G[a:b], out=parts[i])

        ms2 = time_op(spmm_only, args.reps)
        res[f"blocks{nb}"] = {"ms": round(ms, 3), "spmm_only_ms": round(ms2, 3),
                              "edge_GBps": round(bytes_edge / ms / 1e6, 1), "max_abs_diff": err,
                              "G_block_MB": round(N / nb * K * 4 / 1e6, 1)}
        print(f"blocks{nb}", res[f"blocks{nb}"], flush=True)
        del blocks, parts
    print(json.dumps(res))


if __name__ == "__main__":
    main()
