#!/usr/bin/env python
"""The row-partitioned local SpMM per mode: for P = 2, 4, 8, every
rank's block of the World power-law graph (K = 300, all-gathered operand layout) timed in
'ordered' (bitwise scipy), 'fast' (split hub rows) and 'rowwise'; the slowest rank bounds the
step. One GPU plays every rank in turn. HIP events, mean of 10 after 3 warm-ups. A mode
'ordered:256' runs the plan with that task size (whole-workgroup rows past 8 x of it)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphconvgeo_amd import sparse as gs  # noqa: E402
from graphconvgeo_amd.distributed import PartitionPlan, RowPartitionedCSR  # noqa: E402
from graphconvgeo_amd.synth import CONFIGS, synthetic_graph  # noqa: E402

K = 300
dev = torch.device("cuda:0")
cfg = CONFIGS["twitter-world"]
kind = sys.argv[1] if len(sys.argv) > 1 else "powerlaw"
H = synthetic_graph(cfg.n_nodes, cfg.n_edges, kind=kind)


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


for P in [int(x) for x in os.environ.get("PARTS", "1,2,4,8").split(",")]:
    worst = {}
    plan = PartitionPlan(H, P)
    for r in range(P):
        part = RowPartitionedCSR(H, r, P, dev, exchange="allgather", plan=plan)
        operand = gs.empty_dense(part.operand_rows(), K, dev).normal_()
        Y = gs.empty_dense(part.n_local, K, dev)
        line = []
        for mode in os.environ.get("MODES", "ordered,fast,rowwise").split(","):
            m, _, tn = mode.partition(":")  # "ordered:256": the plan's task size
            ms = timed(lambda: gs.spmm(part.A, operand, out=Y, mode=m, task_nnz=int(tn or 0)))
            worst[mode] = max(worst.get(mode, 0.0), ms)
            line.append(f"{mode} {ms:.3f}")
        print(f"{kind} P={P} rank={r} nnz={part.nnz_local} longest={part.A.max_row_nnz()} "
              f"auto={gs.resolve_auto(part.A)} " + " ".join(line), flush=True)
        del part, operand, Y
        torch.cuda.empty_cache()
    print(f"{kind} P={P} slowest rank: " + " ".join(f"{m} {v:.3f}" for m, v in worst.items()),
          flush=True)
