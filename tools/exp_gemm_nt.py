#!/usr/bin/env python
"""NT GEMM (gcg_gemm_nt_f32, LDS-DMA staged) vs the register-B gemm_kernel / LDS-B
gemm_bl_kernel (gcg_gemm_f32) vs hipBLASLt (torch.matmul) on the output-layer shapes:
projection h.W2 (M x 300 x C) and input gradient g.W2^T (M x C x 300). HIP events, mean of
`reps` after a warm-up; sampled rows checked against float64."""
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
    ap.add_argument("--cfgs", default="0;1;2;3;4;5;6;7;8;9;10",
                    help="gcg_gemm_nt f32 tiles")
    ap.add_argument("--shapes", default="840000x300x930,1400000x300x930,840000x930x300,"
                                        "1400000x930x300,450000x300x256,450000x256x300")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    for shp in args.shapes.split(","):
        M, K, N = (int(x) for x in shp.split("x"))
        flop = 2.0 * M * N * K
        A = empty_dense(M, K, dev).copy_(torch.randn((M, K), generator=g, device=dev) * 0.1)
        W = (torch.rand((K, N), generator=g, device=dev) * 2 - 1) * 0.05
        Wp = empty_dense(K, N, dev).copy_(W)          # [K, round4(N)] for gcg_gemm_f32
        Wt = empty_dense(N, K, dev).copy_(W.t())      # [N, round4(K)] for gcg_gemm_nt_f32
        rows = torch.randint(0, M, (512,), generator=g, device=dev)
        ref = (A[rows].double() @ W.double()).cpu().numpy()
        rec = {"shape": f"{M}x{K}x{N}"}
        t = timeit(lambda: torch.matmul(A, W), args.reps)
        rec["hipblaslt"] = round(flop / t / 1e9, 1)
        t = timeit(lambda: dense.gemm(A, Wp), args.reps)
        rec["gemm_f32"] = round(flop / t / 1e9, 1)
        for cfg in args.cfgs.split(";"):  # f32 tiles of gcg_gemm_nt (0..10)
            tile = int(cfg)
            C = dense.gemm_nt(A, Wt, math="f32", tile=tile)
            err = float(np.abs(C[rows].cpu().numpy() - ref).max())
            t = timeit(lambda: dense.gemm_nt(A, Wt, out=C, math="f32", tile=tile), args.reps)
            rec[f"nt[{cfg}]"] = round(flop / t / 1e9, 1)
            rec[f"err[{cfg}]"] = err
        print(json.dumps(rec), flush=True)
        del A, W, Wp, Wt


if __name__ == "__main__":
    main()
