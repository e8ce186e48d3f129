#!/usr/bin/env python
"""NT GEMM products on the bf16 matrix cores (gcg_gemm_nt_f32_bf16x6: three bf16 planes per f32
operand, six plane products) against the f32-MFMA NT kernel (gcg_gemm_nt_f32) on the
output-layer shapes: projection h.W2 (M x 300 x C) and input gradient g.W2^T (M x C x 300).
Tile variants of the pre-split kernel via gcg_gemm_nt's tile argument (1..8); the in-loop split of both operands
(no workspace) as bf16x6_inloop. HIP events, mean of `reps`, interleaved rounds; error on 512
sampled rows against float64, absolute and relative to sum_k |a||b| (the f32 rounding scale)."""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphconvgeo_amd import dense  # noqa: E402
from graphconvgeo_amd.sparse import empty_dense  # noqa: E402


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--cfgs", default="0;1;2;3;4;5;6;7;8",
                    help="gcg_gemm_nt bf16x6 tiles (0 = the default for the shape)")
    ap.add_argument("--shapes", default="840000x300x930,840000x930x300,1400000x300x930,"
                                        "450000x300x256,450000x256x300")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    for shp in args.shapes.split(","):
        M, K, N = (int(x) for x in shp.split("x"))
        flop = 2.0 * M * N * K
        A = empty_dense(M, K, dev).copy_(torch.randn((M, K), generator=g, device=dev) * 0.1)
        W = (torch.rand((K, N), generator=g, device=dev) * 2 - 1) * 0.05
        Wt = empty_dense(N, K, dev).copy_(W.t())
        rows = torch.randint(0, M, (512,), generator=g, device=dev)
        Ar, W64 = A[rows].double().cpu().numpy(), W.double().cpu().numpy()
        ref = Ar @ W64
        scale = np.abs(Ar) @ np.abs(W64)
        C = empty_dense(M, N, dev)
        rec = {"shape": f"{M}x{K}x{N}"}

        def err(C):
            d = np.abs(C[rows].double().cpu().numpy() - ref)
            return float(d.max()), float((d / scale).max())

        variants = [("f32", 0), ("bf16x6_inloop", 0)] + [
            ("bf16x6", int(c)) for c in args.cfgs.split(";") if c]
        for rnd in range(args.rounds):
            for math, cfg in variants:
                key = f"{math}[{cfg}]"
                dense.gemm_nt(A, Wt, out=C, math=math, tile=cfg)
                if rnd == 0:
                    rec[f"err_abs[{key}]"], rec[f"err_rel[{key}]"] = err(C)
                t = timeit(lambda: dense.gemm_nt(A, Wt, out=C, math=math, tile=cfg), args.reps)
                rec.setdefault(f"TF[{key}]", []).append(round(flop / t / 1e9, 1))
        print(json.dumps(rec), flush=True)
        del A, W, Wt, C


if __name__ == "__main__":
    main()
