#!/usr/bin/env python
"""Experiment: does a node relabeling (degree-descending, RCM) raise the gather rate of the
Twitter-World H.Z SpMM? Within-row storage order is kept (bitwise-equal rows, permuted)."""
import os
import sys
import time

import numpy as np
import scipy.sparse as sps
import scipy.sparse.csgraph as csg
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphconvgeo_amd import sparse as gs  # noqa: E402
from graphconvgeo_amd.synth import CONFIGS, synthetic_graph  # noqa: E402
from tools.bench_dense import time_op  # noqa: E402


def relabel(H, perm):
    """H' = P H P^T with row i' = row perm[i'] of H, columns renamed, storage order kept."""
    inv = np.empty_like(perm)
    inv[perm] = np.arange(perm.size)
    lens = np.diff(H.indptr)[perm]
    indptr = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    src = np.concatenate([np.arange(H.indptr[r], H.indptr[r + 1]) for r in perm]) if False else None
    starts = H.indptr[perm].astype(np.int64)
    owner = np.repeat(np.arange(perm.size), lens)
    src = starts[owner] + np.arange(indptr[-1]) - indptr[owner]
    return sps.csr_matrix((H.data[src], inv[H.indices[src]].astype(np.int32), indptr), shape=H.shape)


def main():
    cfg = CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "twitter-world"]
    dev = torch.device("cuda:0")
    H = synthetic_graph(cfg.n_nodes, cfg.n_edges)
    K = 300
    deg = np.diff(H.indptr)
    orders = {"identity": np.arange(H.shape[0]),
              "degree_desc": np.argsort(-deg, kind="stable"),
              "random": np.random.default_rng(1).permutation(H.shape[0])}
    t0 = time.time()
    orders["rcm"] = csg.reverse_cuthill_mckee(H, symmetric_mode=True).astype(np.int64)
    print("rcm s", round(time.time() - t0, 1), flush=True)
    B = 4 * (H.shape[0] + 1) + 8 * H.nnz + 4 * K * H.nnz + 4 * K * H.shape[0]
    Z = torch.randn((H.shape[0], K), device=dev)
    for name, perm in orders.items():
        Hp = relabel(H, perm) if name != "identity" else H
        A = gs.DeviceCSR.from_scipy(Hp, dev, symmetric=True)
        Y = gs.empty_dense(H.shape[0], K, dev)
        for mode in ("ordered", "fast"):
            ms = time_op(lambda: gs.spmm(A, Z, out=Y, mode=mode), 10)
            print(f"{name:12s} {mode:8s} {ms:7.3f} ms  {B / ms / 1e6:8.1f} GB/s", flush=True)
        del A, Y


if __name__ == "__main__":
    main()
