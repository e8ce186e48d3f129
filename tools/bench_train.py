#!/usr/bin/env python
"""BASELINE config 3: Twitter-US-scale 2-layer GCN fwd+bwd (+ Adam) step on one MI355X.

One step = MLPCONV's full-batch epoch (mlpconv.py:293-295): X.W1, H.Z1 (+b1, rectify),
h.W2, (H.Z2 + b2)[train], CE + L1/L2, backward (scatter-add, H.g, h^T.g, g.W2^T, H.g,
X^T.g) and the Lasagne Adam update. Synthetic data (seed 77): power-law graph, 64-nnz/row
BoW X, 60 % of nodes as train indices drawn with replacement (tensormain.py:226).
Prints one JSON line (ms/step, per-SpMM algorithmic bytes summed -> effective GB/s).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from graphconvgeo_amd import sparse as gs  # noqa: E402
from graphconvgeo_amd.mlpconv import LasagneAdam, MLPCONV  # noqa: E402
from graphconvgeo_amd.synth import CONFIGS, synthetic_features, synthetic_graph  # noqa: E402


def spmm_bytes(n_rows, nnz, K):
    return 4 * (n_rows + 1) + 8 * nnz + 4 * K * nnz + 4 * K * n_rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="twitter-us", choices=sorted(CONFIGS))
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--nnz-per-row", type=int, default=64)
    ap.add_argument("--mode", default="auto")
    ap.add_argument("--order", default="auto", choices=["reference", "propagate_first", "auto"],
                    help="layer-2 order (default: MLPCONV's own default, auto)")
    ap.add_argument("--graph", action="store_true", help="replay the step as a captured HIP graph")
    ap.add_argument("--nt-math", default=None, choices=["f32", "bf16x6", "bf16x6_inloop"],
                    help="products of the NT GEMMs (dense.NT_MATH)")
    ap.add_argument("--legacy-stride", action="store_true",
                    help="round-3 row strides for wide operands (sparse.WIDE_ROW_ALIGN = False)")
    ap.add_argument("--inline-weight-grads", action="store_true",
                    help="weight gradients on the main stream (dense.SIDE_STREAM_WEIGHT_GRADS off)")
    ap.add_argument("--inline-head", action="store_true",
                    help="X^T.G dense-head GEMM on the main stream (sparse.TMATMUL_HEAD_SIDE_STREAM off)")
    ap.add_argument("--hybrid-max-cols", type=int, default=None,
                    help="dense-head columns of X^T.g at most (sparse.HYBRID_MAX_COLS)")
    ap.add_argument("--tn-math", default=None, choices=["f32", "bf16x6"],
                    help="products of the weight gradients (dense.TN_MATH)")
    ap.add_argument("--head-math", default=None, choices=["f32", "bf16x6"],
                    help="products of the X^T.g dense-head GEMM (sparse.TMATMUL_HEAD_MATH)")
    ap.add_argument("--side-priority", type=int, default=None,
                    help="priority of the side stream (dense.SIDE_STREAM_PRIORITY; -1 = high)")
    ap.add_argument("--theano-backward", action="store_true",
                    help="reference order: autograd in Theano's association "
                         "(layers.REASSOCIATED_BACKWARD off)")
    args = ap.parse_args()
    gs.WIDE_ROW_ALIGN = not args.legacy_stride
    if args.theano_backward:
        from graphconvgeo_amd import layers
        layers.REASSOCIATED_BACKWARD = False
    from graphconvgeo_amd import dense
    if args.nt_math:
        dense.NT_MATH = args.nt_math
    if args.side_priority is not None:
        dense.SIDE_STREAM_PRIORITY = args.side_priority
    if args.head_math is not None:
        gs.TMATMUL_HEAD_MATH = args.head_math
    if args.tn_math is not None:
        dense.TN_MATH = args.tn_math
    if args.hybrid_max_cols is not None:
        gs.HYBRID_MAX_COLS = args.hybrid_max_cols
    cfg = CONFIGS[args.config]
    dev = torch.device("cuda:0")
    if args.inline_weight_grads:
        from graphconvgeo_amd import dense
        dense.SIDE_STREAM_WEIGHT_GRADS = False
    if args.inline_head:
        gs.TMATMUL_HEAD_SIDE_STREAM = False
    t0 = time.perf_counter()
    H = synthetic_graph(cfg.n_nodes, cfg.n_edges)
    X = synthetic_features(cfg.n_nodes, cfg.n_features, nnz_per_row=args.nnz_per_row)
    t_gen = time.perf_counter() - t0
    n = cfg.n_nodes
    rng = np.random.default_rng(77)
    Y = rng.integers(0, cfg.n_classes, size=n)
    Y[:cfg.n_classes] = np.arange(cfg.n_classes)
    n_tr = int(0.6 * n)
    train = rng.choice(n_tr, size=n_tr).astype(np.int32)
    dev_idx = np.arange(n_tr, int(0.8 * n), dtype=np.int32)
    test_idx = np.arange(int(0.8 * n), n, dtype=np.int32)

    clf = MLPCONV(n_epochs=0, hidden_layer_size=cfg.hidden, device=dev, seed=1, mode=args.mode,
                  order=args.order, use_graph=args.graph)
    clf.fit(X, train, dev_idx, test_idx, Y, H)  # builds layers, uploads H/X, no epochs
    y_train = torch.as_tensor(Y[train].astype(np.int32), device=dev)
    opt = LasagneAdam(clf.params)
    clf.n_epochs = 1  # let _make_train_step capture when --graph
    step = clf._make_train_step(opt, y_train)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / args.steps * 1e3
    K, C = cfg.hidden, cfg.n_classes
    nnzH, nnzX = H.nnz, X.nnz
    # SpMMs per step: X.W1, H.Z1, H.Z2 (train rows only), H.g2, H.g1, X^T.g; the layer-2
    # products are K wide instead of C under the propagate-first order.
    width2 = K if args.order == "propagate_first" or (args.order == "auto" and C > K) else C
    # The layer-2 products run on the distinct targets (RowSelection.distinct) and the backward
    # on (H[targets])^T (sparse.rows_transpose): the targets' nonzeros only, N output rows.
    uniq = np.unique(train)
    nnz_t = int(np.diff(H.indptr)[uniq].sum())
    sp = (spmm_bytes(n, nnzX, K) + spmm_bytes(n, nnzH, K) + spmm_bytes(n, nnz_t, width2) +
          spmm_bytes(n, nnzH, K) + spmm_bytes(cfg.n_features, nnzX, K))
    sp_fwd_rows = spmm_bytes(len(uniq), nnz_t, width2)
    total = sp + sp_fwd_rows
    rec = {"metric": "GCN 2-layer fwd+bwd+adam step", "config": cfg.name, "ms_per_step": round(ms, 3),
           "nodes": n, "nnz_H": nnzH, "nnz_X": nnzX, "F": cfg.n_features, "K": K, "C": C,
           "train_rows": len(train), "train_rows_distinct": int(uniq.size),
           "spmm_algorithmic_bytes_per_step": total,
           "spmm_effective_GBps_if_all_time_in_spmm": round(total / (ms * 1e-3) / 1e9, 1),
           "mode": args.mode, "order": f"{args.order} -> {clf.l_out.order}", "hip_graph": args.graph,
           "inline_weight_grads": args.inline_weight_grads, "inline_head": args.inline_head,
           "legacy_stride": args.legacy_stride, "nt_math": dense.NT_MATH,
           "theano_backward": args.theano_backward, "side_priority": dense.SIDE_STREAM_PRIORITY,
           "head_math": gs.TMATMUL_HEAD_MATH or dense.TN_MATH, "tn_math": dense.TN_MATH,
           "hybrid_max_cols": gs.HYBRID_MAX_COLS,
           "data_gen_s": round(t_gen, 1)}
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
