"""Timings of the SURVEY.md §8f graph-side rows on one MI355X, each beside the reference's
host computation on the same inputs (and checked equal to it):

  normalize   H = D^-1/2 (A+I) D^-1/2 from an undirected edge list
              GPU: graph.normalize_edges_device (gcg_normalize_adjacency_f32; timed with the
                   edge upload, the result left in HBM)
              CPU: graph.normalize_csr -- the tensormain.py:170-180 scipy expression
  spgemm      the input convolution X_conv = H . X (main.py:530, tensormain.py:114)
              GPU: sparse.spgemm (gcg_spgemm_products + gcg_spgemm), operands resident in HBM
              CPU: scipy `H @ X` (csr_matmat, 1 thread) -- the reference's executor
  project     celebrity filter + co-mention projection (data.py:226-250, 364-370)
              GPU: mentions.project_mentions (gcg_project_mention_graph)
              CPU: oracle.project_mentions (pure-Python restatement of the reference's loops)

Prints one JSON line per measurement.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import scipy.sparse as sps
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphconvgeo_amd import sparse as gs  # noqa: E402
from graphconvgeo_amd.graph import normalize_csr, normalize_edges_device  # noqa: E402
from graphconvgeo_amd.synth import CONFIGS, powerlaw_edges, synthetic_graph, synthetic_features  # noqa: E402


def gpu_time(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts))


def emit(rec):
    print(json.dumps(rec), flush=True)


def bench_normalize(cfg, dev, cpu: bool):
    u, v = powerlaw_edges(cfg.n_nodes, cfg.n_edges)
    out = {}
    t_gpu = gpu_time(lambda: out.__setitem__("H", normalize_edges_device(cfg.n_nodes, u, v, dev)))
    rec = {"op": "normalize", "config": cfg.name, "nodes": cfg.n_nodes, "edges": cfg.n_edges,
           "gpu_ms": round(t_gpu * 1e3, 3), "gpu_edges_per_s": round(cfg.n_edges / t_gpu, 1)}
    if cpu:
        adj = sps.csr_matrix((np.ones(len(u)), (u, v)), shape=(cfg.n_nodes, cfg.n_nodes))
        adj = adj + adj.T
        t0 = time.perf_counter()
        Href = normalize_csr(adj)
        t_cpu = time.perf_counter() - t0
        Hg = out["H"].to_scipy()
        rec.update(cpu_s=round(t_cpu, 3), speedup=round(t_cpu / t_gpu, 1),
                   bitwise=bool(np.array_equal(Hg.indptr, Href.indptr) and
                                np.array_equal(Hg.indices, Href.indices) and
                                np.array_equal(Hg.data, Href.data)))
    emit(rec)


def bench_spgemm(cfg, dev, cpu_rows: int):
    H = synthetic_graph(cfg.n_nodes, cfg.n_edges)
    X = synthetic_features(cfg.n_nodes, cfg.n_features)
    Hd = gs.DeviceCSR.from_scipy(H, dev)
    Xd = gs.DeviceCSR.from_scipy(X, dev)
    products = int(np.diff(X.indptr)[H.indices].sum())
    out = {}
    t_gpu = gpu_time(lambda: out.__setitem__("C", gs.spgemm(Hd, Xd)))
    C = out["C"]
    rec = {"op": "spgemm", "config": cfg.name, "nnz_H": int(H.nnz), "nnz_X": int(X.nnz),
           "products": products, "nnz_C": int(C.nnz), "gpu_ms": round(t_gpu * 1e3, 3),
           "gpu_products_per_s": round(products / t_gpu, 1)}
    # CPU: scipy on a row sample (or all rows), compared bitwise with the same GPU rows
    r = min(cpu_rows, H.shape[0]) if cpu_rows > 0 else H.shape[0]
    Hs = H[:r]
    t0 = time.perf_counter()
    Cref = Hs @ X
    t_cpu = time.perf_counter() - t0
    Cref.sort_indices()
    sample_products = int(np.diff(X.indptr)[Hs.indices].sum())
    nnz_r = int(C.indptr[r].item())
    got_ptr = C.indptr[: r + 1].cpu().numpy()
    got_idx = C.indices[:nnz_r].cpu().numpy()
    got_val = C.data[:nnz_r].cpu().numpy()
    rec.update(cpu_rows=r, cpu_products=sample_products, cpu_s=round(t_cpu, 3),
               cpu_products_per_s=round(sample_products / t_cpu, 1),
               speedup_per_product=round((products / t_gpu) / (sample_products / t_cpu), 1),
               bitwise=bool(np.array_equal(got_ptr, Cref.indptr) and np.array_equal(got_idx, Cref.indices)
                            and np.array_equal(got_val, Cref.data.astype(np.float32))))
    emit(rec)


def mention_incidences_synth(n_users, n_mention_only, per_user, seed=7):
    """Synthetic bipartite mention graph: each user mentions `per_user` ids drawn with a
    Zipf-like popularity over users + mention-only names (celebrities appear naturally)."""
    rng = np.random.default_rng(seed)
    n_nodes = n_users + n_mention_only
    pop = np.arange(1, n_nodes + 1, dtype=np.float64) ** -0.6
    pop = pop[rng.permutation(n_nodes)]
    cdf = np.cumsum(pop)
    cdf /= cdf[-1]
    b = np.repeat(np.arange(n_users, dtype=np.int32), per_user)
    a = np.searchsorted(cdf, rng.random(b.size)).clip(0, n_nodes - 1).astype(np.int32)
    return n_users, n_nodes, a, b


def bench_project(n_users, dev, cpu: bool, thr=10):
    from graphconvgeo_amd.mentions import project_mentions
    n_users, n_nodes, a, b = mention_incidences_synth(n_users, n_users // 2, 6)
    out = {}
    t_gpu = gpu_time(lambda: out.__setitem__("e", project_mentions(n_users, n_nodes, a, b, thr, dev)))
    u, v = out["e"]
    rec = {"op": "project", "users": n_users, "nodes": n_nodes, "incidences": int(a.size),
           "edges": int(u.numel()), "gpu_ms": round(t_gpu * 1e3, 3)}
    if cpu:
        from oracle import gcn_oracle as O
        t0 = time.perf_counter()
        ref = O.project_mentions(n_users, n_nodes, a, b, thr)
        t_cpu = time.perf_counter() - t0
        got = np.stack([u.cpu().numpy(), v.cpu().numpy()], axis=1).astype(np.int64)
        rec.update(cpu_s=round(t_cpu, 3), cpu_kind="oracle.project_mentions (Python, 1 thread)",
                   speedup=round(t_cpu / t_gpu, 1), equal=bool(np.array_equal(got, ref)))
    emit(rec)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ops", default="normalize,spgemm,project")
    ap.add_argument("--configs", default="twitter-us,twitter-world")
    ap.add_argument("--spgemm-cpu-rows", type=int, default=60_000,
                    help="rows of H multiplied on the CPU for the scipy baseline (0 = all)")
    args = ap.parse_args()
    dev = torch.device("cuda")
    ops = args.ops.split(",")
    for name in args.configs.split(","):
        cfg = CONFIGS[name]
        if "normalize" in ops:
            bench_normalize(cfg, dev, cpu=True)
        if "spgemm" in ops:
            bench_spgemm(cfg, dev, args.spgemm_cpu_rows)
    if "project" in ops:
        bench_project(20_000, dev, cpu=True)
        bench_project(450_000, dev, cpu=False)


if __name__ == "__main__":
    main()
