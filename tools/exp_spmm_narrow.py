#!/usr/bin/env python
"""Narrow dense widths (K <= 128: the low end of the reference's hidden-size tuning,
tensormain.py:389, and the column shards of the feature-parallel / pipelined multi-GPU forms):
H.Z with 2 or 4 rows per wave (one lane group per row, default) against one row per wave
(GCG_SPMM_SUB=1), World graphs, the mode auto resolves to, interleaved rounds, outputs
compared bitwise. HIP events, mean of 10 after 3 warm-ups; edge-centric GB/s."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphconvgeo_amd import sparse as gs  # noqa: E402
from graphconvgeo_amd.synth import CONFIGS, synthetic_graph  # noqa: E402

dev = torch.device("cuda:0")
cfg = CONFIGS["twitter-world"]
for kind in (sys.argv[1] if len(sys.argv) > 1 else "powerlaw,uniform").split(","):
    H = synthetic_graph(cfg.n_nodes, cfg.n_edges, kind=kind)
    A = gs.DeviceCSR.from_scipy(H, dev, symmetric=True)
    n, nnz = H.shape[0], H.nnz
    mode = gs.resolve_auto(A)
    for K in (16, 32, 64, 76, 96, 128):
        Z = gs.empty_dense(n, K, dev).copy_(torch.randn((n, K), device=dev))
        Y = gs.empty_dense(n, K, dev)
        res, outs = {}, {}
        for rnd in range(3):
            for sub in ("0", "1"):
                os.environ["GCG_SPMM_SUB"] = sub
                for _ in range(3):
                    gs.spmm(A, Z, out=Y, mode=mode)
                if rnd == 0:
                    outs[sub] = Y.clone()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(10):
                    gs.spmm(A, Z, out=Y, mode=mode)
                e.record()
                torch.cuda.synchronize()
                res.setdefault(sub, []).append(round(s.elapsed_time(e) / 10, 3))
        os.environ.pop("GCG_SPMM_SUB", None)
        B = 4 * (n + 1) + 8 * nnz + 4 * K * nnz + 4 * K * n
        print(json.dumps({"graph": kind, "mode": mode, "K": K, "ms_subwave": res["0"],
                          "ms_one_row_per_wave": res["1"],
                          "GBps_subwave": round(B / min(res["0"]) / 1e6, 1),
                          "GBps_one_row": round(B / min(res["1"]) / 1e6, 1),
                          "bitwise": bool(torch.equal(outs["0"], outs["1"]))}), flush=True)
        del Z, Y, outs
        torch.cuda.empty_cache()
    del A
