#!/usr/bin/env python
"""Cost-aware row partition (round 4): for P = 4 and 8 and hub weights
W (distributed.row_partition(hub_weight=W)), every rank's block of the World power-law graph
(K = 300, all-gathered operand layout, 'ordered' = the mode every N runs) timed alone on the one
GPU; prints per-block ms / nnz / hub rows and the slowest-to-mean ratio. HIP events, mean of 10
after 3 warm-ups. Env: PARTS (default 4,8), WEIGHTS (default 1,1.5,2,3), KIND."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphconvgeo_amd import sparse as gs  # noqa: E402
from graphconvgeo_amd.distributed import HUB_ROW_NNZ, RowPartitionedCSR, row_partition  # noqa: E402
from graphconvgeo_amd.synth import CONFIGS, synthetic_graph  # noqa: E402

K = 300
dev = torch.device("cuda:0")
cfg = CONFIGS["twitter-world"]
kind = os.environ.get("KIND", "powerlaw")
H = synthetic_graph(cfg.n_nodes, cfg.n_edges, kind=kind)
lens = np.diff(H.indptr)


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


for P in [int(x) for x in os.environ.get("PARTS", "4,8").split(",")]:
    for w in [float(x) for x in os.environ.get("WEIGHTS", "1,1.5,2,3").split(",")]:
        bounds = row_partition(H.indptr, P, hub_weight=w)
        blocks = []
        for r in range(P):
            part = RowPartitionedCSR(H, r, P, dev, exchange="allgather", bounds=bounds)
            operand = gs.empty_dense(part.operand_rows(), K, dev).normal_()
            Y = gs.empty_dense(part.n_local, K, dev)
            ms = timed(lambda: gs.spmm(part.A, operand, out=Y, mode="ordered"))
            bl = lens[bounds[r]:bounds[r + 1]]
            hub = bl[bl > HUB_ROW_NNZ]
            blocks.append({"rank": r, "ms": round(ms, 4), "nnz": int(bl.sum()),
                           "hub_rows": int(hub.size), "hub_nnz": int(hub.sum()),
                           "longest": int(bl.max())})
            del part, operand, Y
            torch.cuda.empty_cache()
        t = [b["ms"] for b in blocks]
        print(json.dumps({"kind": kind, "P": P, "hub_weight": w, "slowest_ms": max(t),
                          "mean_ms": round(float(np.mean(t)), 4),
                          "slowest_over_mean": round(max(t) / float(np.mean(t)), 4),
                          "blocks": blocks}), flush=True)
