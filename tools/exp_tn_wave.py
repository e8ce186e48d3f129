#!/usr/bin/env python
"""Split-K weight gradient C = A^T.B: per-wave tiles (GCG_TN=MG,NG,PD,0: 64 x 64*NG per wave, one
wave per SIMD) against the default workgroup layout, with the split count swept through
GCG_TN_SLOTS (target tiles per launch). HIP events; every variant's relative error against the
default is printed (a different split count changes the fp32 summation order)."""
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
          (1_400_000, 300, 930, "World dW2 (reference order)"),
          (270_000, 300, 256, "US dW2"),
          (1_400_000, 256, 300, "World X-head^T.dZ1 (as G^T.Xh)")]
variants = os.environ.get("TN_WAVE_VARIANTS",
                          "default;1,2,8,1;1,3,8,0;1,2,8,0;1,3,8,0@1024;1,1,8,4").split(";")


def timed(R, M, N, A, B, reps=3, inner=5):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    r = []
    for _ in range(reps):
        for _ in range(2):
            dense.gemm_tn(A, B)
        s.record()
        for _ in range(inner):
            dense.gemm_tn(A, B)
        e.record()
        torch.cuda.synchronize()
        r.append(round(2.0 * R * M * N / (s.elapsed_time(e) / inner) / 1e9, 1))
    return r


for R, M, N, what in shapes:
    A = empty_dense(R, M, dev).copy_(torch.randn((R, M), generator=g, device=dev))
    B = empty_dense(R, N, dev).copy_(torch.randn((R, N), generator=g, device=dev))
    ref64 = (A[:, :M].double().T @ B[:, :N].double())
    res = {}
    for rnd in range(2):  # interleaved rounds
        for v in variants:
            os.environ.pop("GCG_TN", None)
            os.environ.pop("GCG_TN_SLOTS", None)
            if v != "default":
                tile, _, slots = v.partition("@")
                os.environ["GCG_TN"] = tile
                if slots:
                    os.environ["GCG_TN_SLOTS"] = slots
            out = dense.gemm_tn(A, B).clone()
            err = float(((out.double() - ref64).abs() / (ref64.abs() + 1.0)).max())
            res.setdefault(v, {"TFLOPs": [], "rel_err_vs_f64": err})["TFLOPs"] += timed(R, M, N, A, B)
    os.environ.pop("GCG_TN", None)
    os.environ.pop("GCG_TN_SLOTS", None)
    print(json.dumps({"shape": f"{R}x{M}x{N}", "what": what, "res": res}), flush=True)
    del A, B, ref64
    torch.cuda.empty_cache()
