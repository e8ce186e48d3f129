#!/usr/bin/env python
"""The Xt . dZ1 tail gather of the W1 gradient (DeviceCSR.tmatmul: CSR(X^T) without the dense
Zipf-head columns, mlpconv.py:71's gradient) alone at a config's size, per SpMM mode and task
size; HIP events, mean of 10 after 3 warm-ups, 2 interleaved rounds."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphconvgeo_amd import sparse as gs  # noqa: E402
from graphconvgeo_amd.synth import CONFIGS, synthetic_features  # noqa: E402

dev = torch.device("cuda:0")
cfg = CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "twitter-world"]
K = cfg.hidden
X = synthetic_features(cfg.n_nodes, cfg.n_features, nnz_per_row=64)
A = gs.DeviceCSR.from_scipy(X, dev)
cols, Xh, tail_t = A._dense_column_split()
G = gs.empty_dense(cfg.n_nodes, K, dev).normal_()
rec = {"config": cfg.name, "tail_nnz": tail_t.nnz, "tail_rows": tail_t.n_rows,
       "tail_max_row": tail_t.max_row_nnz(), "head_cols": int(cols.numel()),
       "auto": gs.resolve_auto(tail_t)}
forms = [("auto", 0), ("rowwise", 0)] + [(m, t) for m in ("ordered", "fast") for t in (0, 64, 256, 512)]
out = gs.empty_dense(tail_t.n_rows, K, dev)
for rnd in range(2):
    for mode, t in forms:
        f = lambda: gs.spmm(tail_t, G, mode=mode, out=out, task_nnz=t)  # noqa: E731
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(10):
            f()
        e.record()
        torch.cuda.synchronize()
        rec.setdefault(f"{mode}:{t}", []).append(round(s.elapsed_time(e) / 10, 3))
print(json.dumps(rec), flush=True)
