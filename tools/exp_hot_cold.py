#!/usr/bin/env python
"""Gather hint (DeviceCSR.gather_hint, gcg_spmm_csr_f32_planned_hint): the rows of all but the
most frequent columns of H are gathered with non-temporal loads so the hub rows stay in the
L2 / Infinity Cache. Hot-set sizes (sparse.GATHER_HINT_HOT_BYTES) against no hint
(GCG_SPMM_NO_HINT=1), H.Z at K = 300 on the Twitter-World and Twitter-US graphs, the mode auto
resolves to, interleaved rounds, outputs compared bitwise. HIP events, mean of 10."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphconvgeo_amd import sparse as gs  # noqa: E402
from graphconvgeo_amd.synth import CONFIGS, synthetic_graph  # noqa: E402

dev = torch.device("cuda:0")
gs.GATHER_HINT = True
if os.environ.get("HINT_MIN_TABLE_MB"):
    gs.GATHER_HINT_MIN_TABLE = int(os.environ["HINT_MIN_TABLE_MB"]) << 20
K = int(os.environ.get("HINT_K", "300"))
sizes_mb = [int(x) for x in os.environ.get("HINT_MB", "8,16,32,64").split(",")]
for spec in (sys.argv[1] if len(sys.argv) > 1 else "twitter-world:powerlaw,twitter-us:powerlaw,"
             "twitter-world:uniform").split(","):
    name, kind = spec.split(":")
    cfg = CONFIGS[name]
    H = synthetic_graph(cfg.n_nodes, cfg.n_edges, kind=kind)
    n, nnz = H.shape[0], H.nnz
    A = gs.DeviceCSR.from_scipy(H, dev, symmetric=True)
    mode = gs.resolve_auto(A)
    Z = gs.empty_dense(n, K, dev).copy_(torch.randn((n, K), device=dev))
    Y = gs.empty_dense(n, K, dev)
    os.environ["GCG_SPMM_NO_HINT"] = "1"
    ref = gs.spmm(A, Z, mode=mode).clone()

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
    res, used = {}, {}
    for rnd in range(3):
        os.environ["GCG_SPMM_NO_HINT"] = "1"
        res.setdefault("no hint", []).append(timed())
        os.environ.pop("GCG_SPMM_NO_HINT", None)
        for mb in sizes_mb:
            gs.GATHER_HINT_HOT_BYTES = mb << 20
            used[mb] = A.gather_hint(4 * min(Z.stride(0), 512)) is not None
            res.setdefault(f"hot {mb} MB", []).append(timed())
            assert torch.equal(Y, ref), f"hint {mb} MB changed the result"
    gs.GATHER_HINT_HOT_BYTES = 32 << 20
    B = 4 * (n + 1) + 8 * nnz + 4 * K * nnz + 4 * K * n
    print(json.dumps({"graph": spec, "mode": mode, "K": K, "ms": res, "hint_used": used,
                      "GBps_no_hint": round(B / min(res["no hint"]) / 1e6, 1),
                      "GBps_32MB": round(B / min(res.get("hot 32 MB", [1e9])) / 1e6, 1)}), flush=True)
    del A, Z, Y, ref
    torch.cuda.empty_cache()
