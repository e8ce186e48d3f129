#!/usr/bin/env python
"""Split-K weight gradient C = A^T . B (gcg_gemm_tn_f32) with f32 MFMA products against the
bf16x6 tiles (gemm_tn6_kernel, GCG_TN_MATH=bf16x6): dW2 = P^T . G at Twitter-World's and
Twitter-US's shapes. HIP events, mean of 10, interleaved rounds; error on the whole output
against float64, max |err| / (sum_r |a||b|). The kernel and knob were reverted after this A/B (no gain:
profiles/r04/tn_bf16x6_ab.jsonl); they live in commit decb56f."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphconvgeo_amd import dense  # noqa: E402
from graphconvgeo_amd.sparse import empty_dense  # noqa: E402


def timeit(fn, reps=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(3)
for R, M, N in ((840_000, 300, 930), (1_400_000, 300, 930), (270_000, 300, 256)):
    A = empty_dense(R, M, dev).copy_(torch.randn((R, M), generator=g, device=dev) * 0.1)
    B = empty_dense(R, N, dev).copy_(torch.randn((R, N), generator=g, device=dev) * 0.01)
    ref = (A.double().t() @ B.double())
    scl = (A.double().abs().t() @ B.double().abs())
    rec = {"shape": f"{R}x{M}x{N}"}
    flops = 2.0 * R * M * N
    for rnd in range(2):
        for math in ("f32", "bf16x6"):
            os.environ["GCG_TN_MATH"] = math
            C = dense.gemm_tn(A, B)
            if rnd == 0:
                rec[f"err_rel[{math}]"] = float(((C.double() - ref).abs() / scl).max())
            ms = timeit(lambda: dense.gemm_tn(A, B))
            rec.setdefault(f"TF[{math}]", []).append(round(flops / ms / 1e9, 1))
    os.environ.pop("GCG_TN_MATH", None)
    print(json.dumps(rec), flush=True)
    del A, B, ref, scl
    torch.cuda.empty_cache()
