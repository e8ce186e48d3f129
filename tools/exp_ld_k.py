#!/usr/bin/env python
"""Row stride of the dense operand for the reference's other hidden sizes (tensormain.py:
default 500, 1500): H.Z with Z / Y as [n, ld] buffers viewed [n, K], ld swept, interleaved rounds
on one device. sparse.row_stride picks the stride (K = 300 -> 304: every gathered row on exactly
10 lines); at K = 500 / 1500 no non-multiple of 128 B keeps rows on the fewest lines, so it
falls back to round4(K). HIP events, mean of 10 after 3 warm-ups."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphconvgeo_amd import sparse as gs  # noqa: E402
from graphconvgeo_amd.synth import CONFIGS, synthetic_graph  # noqa: E402

dev = torch.device("cuda:0")
cfg = CONFIGS["twitter-world"]
cases = {300: [300, 304, 320], 500: [500, 504, 512, 528], 1500: [1500, 1504, 1536]}
if os.environ.get("LD_CASES"):  # e.g. "930:932,936,944,960;928:928"
    cases = {int(k): [int(x) for x in v.split(",")]
             for k, v in (c.split(":") for c in os.environ["LD_CASES"].split(";"))}
for kind in (sys.argv[1] if len(sys.argv) > 1 else "powerlaw,uniform").split(","):
    H = synthetic_graph(cfg.n_nodes, cfg.n_edges, kind=kind)
    A = gs.DeviceCSR.from_scipy(H, dev, symmetric=True)
    n, nnz = H.shape[0], H.nnz
    mode = gs.resolve_auto(A)
    for K, lds in cases.items():
        bufs = {}
        src = torch.randn((n, K), device=dev)
        for ld in lds:
            Zb = torch.empty((n, ld), device=dev)
            Zb[:, :K].copy_(src)
            bufs[ld] = (Zb[:, :K], torch.empty((n, ld), device=dev)[:, :K])
        ref = gs.spmm(A, bufs[lds[0]][0], mode=mode).clone()
        res = {}
        for rnd in range(3):
            for ld, (Z, Y) in bufs.items():
                for _ in range(3):
                    gs.spmm(A, Z, out=Y, mode=mode)
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(10):
                    gs.spmm(A, Z, out=Y, mode=mode)
                e.record()
                torch.cuda.synchronize()
                res.setdefault(ld, []).append(round(s.elapsed_time(e) / 10, 3))
                if rnd == 0:
                    assert torch.equal(Y, ref), "stride changed the result"
        print(json.dumps({"graph": kind, "mode": mode, "K": K, "row_stride_now": gs.row_stride(K),
                          "ms_by_ld": res}), flush=True)
        del bufs, ref, src
        torch.cuda.empty_cache()
    del A
