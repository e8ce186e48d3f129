#!/usr/bin/env python
"""Experiment: dW1 = X^T . G (grad of S.dot(X, W1), mlpconv.py:71) with the most frequent
bag-of-words features taken out of the gather: X = X_head + X_tail, where X_head holds the Fh
most frequent columns as a dense N x Fh matrix. dW1[head] = X_head^T . G runs on the split-K
MFMA GEMM (reads G once), dW1[tail] = X_tail^T . G stays a CSR gather SpMM. With Zipf word
frequencies the head holds ~half the nonzeros. Twitter-World shapes, HIP events."""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from graphconvgeo_amd import dense, sparse as gs  # noqa: E402
from graphconvgeo_amd.synth import CONFIGS, synthetic_features  # noqa: E402
from tools.exp_xtg_blocks import time_op  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="twitter-world")
    ap.add_argument("--heads", default="64,128,192,256,384")
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    cfg = CONFIGS[args.config]
    dev = torch.device("cuda:0")
    X = synthetic_features(cfg.n_nodes, cfg.n_features, nnz_per_row=64)
    N, F, K = cfg.n_nodes, cfg.n_features, cfg.hidden
    Xd = gs.DeviceCSR.from_scipy(X, dev)
    G = gs.empty_dense(N, K, dev)
    G.copy_(torch.randn((N, K), device=dev))
    ref = gs.spmm(Xd.transpose(), G)
    res = {"single_ms": round(time_op(lambda: gs.spmm(Xd.transpose(), G, out=ref), args.reps), 3)}
    print(res, flush=True)
    freq = np.bincount(X.indices, minlength=F)
    order = np.argsort(-freq, kind="stable")
    rows = np.repeat(np.arange(N, dtype=np.int64), np.diff(X.indptr))
    for fh in [int(x) for x in args.heads.split(",")]:
        head = np.sort(order[:fh])
        slot = np.full(F, -1, np.int64)
        slot[head] = np.arange(fh)
        s = slot[X.indices]
        m = s >= 0
        Xh = torch.zeros((N, (fh + 3) // 4 * 4), device=dev)
        Xh[torch.as_tensor(rows[m], device=dev), torch.as_tensor(s[m], device=dev)] = \
            torch.as_tensor(X.data[m], device=dev)
        Xh = Xh[:, :fh]
        Xt = X.copy()
        Xt.data = np.where(m, 0, X.data).astype(np.float32)
        Xt.eliminate_zeros()
        Ttail = gs.DeviceCSR.from_scipy(Xt, dev).transpose()
        head_t = torch.as_tensor(head, device=dev)
        out = gs.empty_dense(F, K, dev)

        def run():
            gs.spmm(Ttail, G, out=out)
            out.index_copy_(0, head_t, dense.gemm_tn(Xh, G))
            return out

        run()
        err = float((out - ref).abs().max())
        scale = float(ref.abs().max())
        ms = time_op(run, args.reps)
        ms_tail = time_op(lambda: gs.spmm(Ttail, G, out=out), args.reps)
        ms_head = time_op(lambda: dense.gemm_tn(Xh, G), args.reps)
        r = {"ms": round(ms, 3), "tail_ms": round(ms_tail, 3), "head_ms": round(ms_head, 3),
             "head_nnz_frac": round(float(m.mean()), 3), "max_abs_diff": err, "max_abs": scale}
        res[f"head{fh}"] = r
        print(f"head{fh}", r, flush=True)
        del Xh, Ttail, Xt
    print(json.dumps(res))


if __name__ == "__main__":
    main()
