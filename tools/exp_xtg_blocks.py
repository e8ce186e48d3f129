#!/usr/bin/env python
"""X^T . G (the W1 gradient, grad of mlpconv.py:71) with the contraction rows blocked so each
block's G rows fit the 256 MB Infinity Cache: the tail CSR(X_tail^T) split by document ranges
[i_b, i_b+1), one SpMM per block into its own partial (timing only; a bitwise form would continue
each feature row's storage-order sum from the previous block's output). Compared with the one
unblocked tail launch, alone and with the dense-head product X_head^T . G beside it on a side
stream as in DeviceCSR.tmatmul. HIP events, interleaved."""
import json
import os
import sys

import numpy as np
import scipy.sparse as sps
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphconvgeo_amd import dense  # noqa: E402
from graphconvgeo_amd import sparse as gs  # noqa: E402
from graphconvgeo_amd.synth import CONFIGS, synthetic_features  # noqa: E402

dev = torch.device("cuda:0")
K = 300


def timed(fn, reps=10):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return round(s.elapsed_time(e) / reps, 3)


for name in (sys.argv[1] if len(sys.argv) > 1 else "twitter-us,twitter-world").split(","):
    cfg = CONFIGS[name]
    X = synthetic_features(cfg.n_nodes, cfg.n_features, nnz_per_row=64)
    n = X.shape[0]
    A = gs.DeviceCSR.from_scipy(X, dev)
    cols, Xh, tail_t = A._dense_column_split()
    G = gs.empty_dense(n, K, dev).copy_(torch.randn((n, K), device=dev))
    # host copy of the tail transpose, sliced by document (column) ranges
    T = sps.csr_matrix((tail_t.data.cpu().numpy(), tail_t.indices.cpu().numpy(),
                        tail_t.indptr.cpu().numpy()), shape=tail_t.shape)
    rec = {"config": name, "nnz_X": int(X.nnz), "nnz_tail": int(T.nnz), "head_cols": int(cols.numel()),
           "G_MB": round(n * 304 * 4 / 2**20, 1)}
    side = torch.cuda.Stream(device=dev)
    variants = {}
    for nb in (1, 2, 3, 4, 6, 8, 12):
        bounds = np.linspace(0, n, nb + 1).astype(np.int64)
        blocks = [gs.DeviceCSR.from_scipy(T[:, bounds[b]:bounds[b + 1]].tocsr(), dev)
                  for b in range(nb)]
        outs = [gs.empty_dense(T.shape[0], K, dev) for _ in range(nb)]
        Gs = [G[bounds[b]:bounds[b + 1]] for b in range(nb)]
        variants[nb] = (blocks, outs, Gs)
    res = {}
    for rnd in range(2):
        for nb, (blocks, outs, Gs) in variants.items():
            def tail():
                for Bk, o, g in zip(blocks, outs, Gs):
                    gs.spmm(Bk, g, out=o, mode="fast")

            def both():
                side.wait_stream(torch.cuda.current_stream(dev))
                with torch.cuda.stream(side):
                    dense.gemm_tn(Xh, G)
                tail()
                torch.cuda.current_stream(dev).wait_stream(side)
            res.setdefault(f"tail x{nb}", []).append(timed(tail))
            res.setdefault(f"tail x{nb} + head", []).append(timed(both))
    res["head alone"] = [timed(lambda: dense.gemm_tn(Xh, G))]
    print(json.dumps({**rec, "ms": res}), flush=True)
    del A, G, variants, Xh, tail_t
    torch.cuda.empty_cache()
