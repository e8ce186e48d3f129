#!/usr/bin/env python
"""X . W1 (mlpconv.py:71; W1 cache-resident) per SpMM mode / task size at a config's size, after
round 5's 128-nonzero ordered plans: 'auto' picks the plan-less rowwise form for X (no hub rows).
HIP events, mean of 10 after 3 warm-ups, 2 interleaved rounds."""
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
W = gs.empty_dense(cfg.n_features, K, dev).normal_()
out = gs.empty_dense(cfg.n_nodes, K, dev)
rec = {"config": cfg.name, "auto": gs.resolve_auto(A), "nnz": A.nnz, "longest": A.max_row_nnz()}
forms = [("rowwise", 0), ("ordered", 0), ("ordered", 64), ("ordered", 256), ("ordered", 512)]
for rnd in range(2):
    for mode, t in forms:
        f = lambda: gs.spmm(A, W, mode=mode, out=out, task_nnz=t)  # noqa: E731
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
