"""Experiment: does gathering from an Infinity-Cache-sized slice of the dense operand beat
gathering from the whole 1.68 GB operand?  (Motivation: Xᵀ·G at Twitter-World gathers one
1200-B row of G per nonzero from HBM; row-blocking X so each pass gathers from a ~150 MB slice
of G would keep the slice in the 256 MiB Infinity Cache.)

Random CSR with `rows` output rows and `nnz` nonzeros, column ids uniform in [0, R), K = 300.
Reports ms and edge-centric GB/s for R = full (1.4M rows) and for MALL-sized slices, both for
the whole nnz (one pass) and nnz / passes (one slice pass, scaled by passes).
"""
import argparse
import json

import numpy as np
import scipy.sparse as sps
import torch
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphconvgeo_amd import sparse as gs


def rand_csr(rows, cols, nnz, rng):
    r = np.sort(rng.integers(0, rows, nnz)).astype(np.int32)
    c = rng.integers(0, cols, nnz).astype(np.int32)
    m = sps.csr_matrix((np.ones(nnz, np.float32), (r, c)), shape=(rows, cols))
    m.sum_duplicates()
    m.sort_indices()
    return m


def timeit(fn, reps=10):
    for _ in range(3):
        fn()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in evs:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in evs]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=50_000)
    ap.add_argument("--nnz", type=int, default=45_000_000)
    ap.add_argument("--n", type=int, default=1_400_000)
    ap.add_argument("--K", type=int, default=300)
    args = ap.parse_args()
    rng = np.random.default_rng(1)
    dev = torch.device("cuda")
    K = args.K
    G = torch.randn((args.n, K), device=dev)
    out = gs.empty_dense(args.rows, K, dev)
    res = []
    for R in [args.n, 500_000, 250_000, 125_000, 62_500, 31_250]:
        passes = max(1, args.n // R)
        nnz = args.nnz // passes
        A = gs.DeviceCSR.from_scipy(rand_csr(args.rows, R, nnz, rng), dev)
        Zs = G[:R]
        ms = timeit(lambda: gs.spmm(A, Zs, out=out, mode="fast"))
        b = 8 * A.nnz + 4 * K * A.nnz + 4 * K * args.rows
        rec = {"R": R, "slice_MB": round(R * K * 4 / 1e6, 1), "passes": passes, "nnz_pass": int(A.nnz),
               "ms_pass": round(ms, 4), "ms_total": round(ms * passes, 3),
               "edge_GBps": round(b / ms / 1e6, 1)}
        print(json.dumps(rec), flush=True)
        res.append(rec)
        del A


if __name__ == "__main__":
    main()
