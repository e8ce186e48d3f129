#!/usr/bin/env python
"""Three-tier gather hint (experiment): hot columns gathered with the default policy, a warm
tier (sparse.GATHER_HINT_WARM_*, bit 30) with the load policy GCG_SPMM_WARM_POL, the rest
non-temporal -- against no hint and the two-tier hint. H.Z at K = 300 on the Twitter-World
(power-law, uniform) and Twitter-US graphs in the mode auto resolves to, interleaved rounds,
outputs compared bitwise. HIP events, mean of 10 launches. The knobs it drives were reverted
after the A/B (profiles/r04/hint_tiers.jsonl: slower under every policy); they live in commit 1259152."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphconvgeo_amd import sparse as gs  # noqa: E402
from graphconvgeo_amd.synth import CONFIGS, synthetic_graph  # noqa: E402

dev = torch.device("cuda:0")
K = 300
warm_mb = [int(x) for x in os.environ.get("WARM_MB", "96,192").split(",")]
pols = [int(x) for x in os.environ.get("WARM_POL", "0,1,16,17").split(",")]
ENV = ("GCG_SPMM_NO_HINT", "GCG_SPMM_HINT_TIERS", "GCG_SPMM_WARM_POL")


def setenv(**kw):
    for k in ENV:
        os.environ.pop(k, None)
    for k, v in kw.items():
        os.environ[k] = str(v)


for spec in (sys.argv[1] if len(sys.argv) > 1 else
             "twitter-world:powerlaw,twitter-us:powerlaw,twitter-world:uniform").split(","):
    name, kind = spec.split(":")
    cfg = CONFIGS[name]
    H = synthetic_graph(cfg.n_nodes, cfg.n_edges, kind=kind)
    n, nnz = H.shape[0], H.nnz
    A = gs.DeviceCSR.from_scipy(H, dev, symmetric=True)
    mode = gs.resolve_auto(A)
    Z = gs.empty_dense(n, K, dev).copy_(torch.randn((n, K), device=dev))
    Y = gs.empty_dense(n, K, dev)
    setenv(GCG_SPMM_NO_HINT=1)
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
        assert torch.equal(Y, ref), "hint changed the result"
        return round(s.elapsed_time(e) / 10, 3)

    res, warm_rows = {}, {}
    for rnd in range(3):
        setenv(GCG_SPMM_NO_HINT=1)
        res.setdefault("no hint", []).append(timed())
        setenv()
        res.setdefault("2 tiers", []).append(timed())
        for mb in warm_mb:
            gs.GATHER_HINT_WARM_BYTES = mb << 20
            A.__dict__.get("_gather_hints", {}).pop((gs.GATHER_HINT_HOT_BYTES // 1216, 3), None)
            for pol in pols:
                setenv(GCG_SPMM_HINT_TIERS=3, GCG_SPMM_WARM_POL=pol)
                res.setdefault(f"warm {mb} MB pol {pol}", []).append(timed())
                warm_rows[mb] = getattr(A, "_hint_warm_rows", None)
    B = 4 * (n + 1) + 8 * nnz + 4 * K * nnz + 4 * K * n
    best = {k: min(v) for k, v in res.items()}
    print(json.dumps({"graph": spec, "mode": mode, "K": K, "ms_min": best, "ms": res,
                      "hot_rows": getattr(A, "_hint_hot_rows", None), "warm_rows": warm_rows,
                      "GBps": {k: round(B / v / 1e6, 1) for k, v in best.items()}}), flush=True)
    del A, Z, Y, ref
    torch.cuda.empty_cache()
