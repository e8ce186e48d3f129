#!/usr/bin/env python
"""Split-K weight gradient C = A^T.B: wave layout along N (WM = 1, the round-2 default) vs WM
waves stacked along M (GCG_TN=MG,NG,PD,WM), at the training step's shapes. HIP events, mean of
5 launches x 3; every variant compared with the default (different split counts: fp32 rounding)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphconvgeo_amd import dense  # noqa: E402
from graphconvgeo_amd.sparse import empty_dense  # noqa: E402

dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
shapes = [(840_000, 300, 930, "World dW2 (propagate-first)"),
          (270_000, 300, 256, "US dW2"),
          (1_400_000, 256, 300, "World X-head^T.dZ1 (as G^T.Xh: 1.4M x 300 x 256)")]
variants = os.environ.get("TN_VARIANTS", "default,1,2,8,5,1,1,8,5,1,2,8,4,1,1,8,4").split(",")
names = ["default"] + [",".join(variants[i:i + 4]) for i in range(1, len(variants), 4)]
for R, M, N, what in shapes:
    A = empty_dense(R, M, dev).copy_(torch.randn((R, M), generator=g, device=dev))
    B = empty_dense(R, N, dev).copy_(torch.randn((R, N), generator=g, device=dev))
    ref, res = None, {}
    for v in names:
        if v == "default":
            os.environ.pop("GCG_TN", None)
        else:
            os.environ["GCG_TN"] = v
        out = dense.gemm_tn(A, B).clone()
        err = 0.0 if ref is None else float(((out - ref).abs() / (ref.abs() + 1.0)).max())
        ref = out if ref is None else ref
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        r = []
        for _ in range(3):
            for _ in range(2):
                dense.gemm_tn(A, B)
            s.record()
            for _ in range(5):
                dense.gemm_tn(A, B)
            e.record()
            torch.cuda.synchronize()
            r.append(round(2.0 * R * M * N / (s.elapsed_time(e) / 5) / 1e9, 1))
        res[v] = {"TFLOPs": r, "rel_err_vs_default": err}
    os.environ.pop("GCG_TN", None)
    print(json.dumps({"shape": f"{R}x{M}x{N}", "what": what, "res": res}), flush=True)
    del A, B
