#!/usr/bin/env python
"""Column-sliced hub rows (round 5, spmm.hip coop_slice: ordered plan 1) vs every long row
on one workgroup (ordered plan 2) vs split rows (fast): (1) one hub row of L nonzeros alone
against a Twitter-World-sized Z (1.4M x 300); (2) the World row blocks of a P-way partition
(default P = 8, ranks 0 and 1); (3) the whole World graph. HIP events, mean of 10 after 3
warm-ups; the results bitwise-checked between the two ordered plans."""
import json
import os
import sys

import numpy as np
import scipy.sparse as sps
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphconvgeo_amd import sparse as gs  # noqa: E402
from graphconvgeo_amd.distributed import PartitionPlan, RowPartitionedCSR  # noqa: E402
from graphconvgeo_amd.synth import CONFIGS, synthetic_graph  # noqa: E402

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
    return s.elapsed_time(e) / reps


def run(A, Z, Y, task_nnz=0):
    out = {}
    res = {}
    for name, ordered in (("sliced", 1), ("one_wg", 2)):
        gs.ORDERED_PLAN = ordered
        out[name] = round(timed(lambda: gs.spmm(A, Z, out=Y, mode="ordered", task_nnz=task_nnz)), 4)
        res[name] = Y.clone()
    gs.ORDERED_PLAN = 1
    out["hub_rows"] = A.plan(None, 1, task_nnz).info()["n_sliced_rows"]
    out["fast"] = round(timed(lambda: gs.spmm(A, Z, out=Y, mode="fast", task_nnz=task_nnz)), 4)
    out["bitwise"] = bool(torch.equal(res["sliced"], res["one_wg"]))
    return out


n = 1_400_000
Z = gs.empty_dense(n, K, dev).normal_()
for L in [int(x) for x in os.environ.get("HUB_LENS", "12000,24000").split(",")]:
    rng = np.random.default_rng(L)
    lens = np.full(4000, 8)
    lens[0] = L
    indptr = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    idx = rng.integers(0, n, indptr[-1]).astype(np.int32)
    H = sps.csr_matrix((rng.random(idx.size).astype(np.float32), idx, indptr), shape=(4000, n))
    A = gs.DeviceCSR.from_scipy(H, dev)
    Y = gs.empty_dense(4000, K, dev)
    for tn in [int(x) for x in os.environ.get("TASKS", "128,512").split(",")]:
        print(json.dumps({"case": "one hub row", "L": L, "task_nnz": tn, **run(A, Z, Y, tn)}),
              flush=True)
    del A, Y
cfg = CONFIGS["twitter-world"]
Hw = synthetic_graph(cfg.n_nodes, cfg.n_edges)
P = int(os.environ.get("P", "8"))
plan = PartitionPlan(Hw, P)
for r in [int(x) for x in os.environ.get("RANKS", "0,1").split(",")]:
    part = RowPartitionedCSR(Hw, r, P, dev, exchange="allgather", plan=plan)
    operand = gs.empty_dense(part.operand_rows(), K, dev).normal_()
    Y = gs.empty_dense(part.n_local, K, dev)
    print(json.dumps({"case": f"World P={P} block", "rank": r, "nnz": part.nnz_local,
                      **run(part.A, operand, Y)}), flush=True)
    del part, operand, Y
    torch.cuda.empty_cache()
A = gs.DeviceCSR.from_scipy(Hw, dev, symmetric=True)
Zw = gs.empty_dense(Hw.shape[0], K, dev).normal_()
Y = gs.empty_dense(Hw.shape[0], K, dev)
print(json.dumps({"case": "World whole graph", "nnz": int(Hw.nnz), **run(A, Zw, Y)}), flush=True)
