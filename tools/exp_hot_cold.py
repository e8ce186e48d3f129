#!/usr/bin/env python
"""Experiment: keep the hub rows of Z in the L2 by gathering every other row with a
non-temporal load (GCG_SPMM_HC=1: the kernel reads a cold-column sign bit from the indices).
On the power-law World graph ~40 % of the gathers hit the top ~2,000 rows (2.4 MB, inside one
XCD's 4 MB L2), yet L2->fabric bytes are 0.95x the edge-centric count. Hot set = the N most
frequent columns; N = 0 (all cold) and N = n (all hot: the branch alone) bracket it.
HIP events, interleaved rounds, outputs compared bitwise with the default kernel."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphconvgeo_amd import sparse as gs  # noqa: E402
from graphconvgeo_amd.synth import CONFIGS, synthetic_graph  # noqa: E402

dev = torch.device("cuda:0")
cfg = CONFIGS["twitter-world"]
K = 300
for kind in (sys.argv[1] if len(sys.argv) > 1 else "powerlaw").split(","):
    H = synthetic_graph(cfg.n_nodes, cfg.n_edges, kind=kind)
    n, nnz = H.shape[0], H.nnz
    A = gs.DeviceCSR.from_scipy(H, dev, symmetric=True)
    mode = gs.resolve_auto(A)
    Z = gs.empty_dense(n, K, dev).copy_(torch.randn((n, K), device=dev))
    Y = gs.empty_dense(n, K, dev)
    ref = gs.spmm(A, Z, mode=mode).clone()
    orig = A.indices.clone()
    counts = np.bincount(H.indices, minlength=n)
    order = np.argsort(-counts, kind="stable")
    variants = {}
    for nh in (0, 1000, 2000, 3000, 6000, 12000, n):
        hot = np.zeros(n, dtype=bool)
        hot[order[:nh]] = True
        share = float(counts[hot].sum() / nnz)
        cold_bit = torch.as_tensor(~hot, device=dev)[orig.long()]
        flagged = torch.where(cold_bit, orig | torch.tensor(-2**31, dtype=torch.int32, device=dev), orig)
        variants[nh] = (flagged, share)
    B = 4 * (n + 1) + 8 * nnz + 4 * K * nnz + 4 * K * n

    def timed():
        for _ in range(3):
            gs.spmm(A, Z, out=Y, mode=mode)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(10):
            gs.spmm(A, Z, out=Y, mode=mode)
        e.record()
        torch.cuda.synchronize()
        return round(s.elapsed_time(e) / 10, 3)
    res = {}
    for rnd in range(3):
        os.environ.pop("GCG_SPMM_HC", None)
        A.indices.copy_(orig)
        res.setdefault("default", []).append(timed())
        for nh, (flagged, share) in variants.items():
            A.indices.copy_(flagged)
            os.environ["GCG_SPMM_HC"] = "1"
            t = timed()
            ok = bool(torch.equal(Y, ref))
            os.environ.pop("GCG_SPMM_HC", None)
            res.setdefault(f"hot={nh} ({share:.2f} of nnz)", []).append(t)
            assert ok, f"hot={nh}: result differs"
    A.indices.copy_(orig)
    print(json.dumps({"graph": kind, "mode": mode, "ms": res,
                      "GBps_default": round(B / min(res["default"]) / 1e6, 1)}), flush=True)
    del A, Z, Y, ref
    torch.cuda.empty_cache()
