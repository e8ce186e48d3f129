#!/usr/bin/env python
"""bf16x6 NT GEMM tiles (gcg_gemm_nt_f32 math=bf16x6, tile=0 default / 1..N) at the output
layer's Twitter-World shapes: projection P.W2 + b2 (840k x 300 x 930) and input gradient
dP = G.W2^T (840k x 930 x 300). HIP events, mean of `reps` after 3 warm-ups, the tiles
alternated for `rounds`; every tile's output compared bit for bit with tile 0's (the bf16x6
tiles compute the same products in the same order).

  python tools/exp_nt_tiles.py --tiles 0,9,10 --rounds 3
"""
import argparse
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphconvgeo_amd import dense  # noqa: E402
from graphconvgeo_amd.sparse import empty_dense  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tiles", default="0,9,10")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(5)
    T, K, C = 840_000, 300, 930
    P = empty_dense(T, K, dev).copy_(torch.randn((T, K), generator=g, device=dev) * 0.1)
    W = (torch.rand((K, C), generator=g, device=dev) * 2 - 1) * math.sqrt(6.0 / (K + C))
    b = torch.randn(C, generator=g, device=dev) * 0.01
    G = empty_dense(T, C, dev).copy_(torch.randn((T, C), generator=g, device=dev) * 1e-3)
    W_ck = dense._WeightCache().get(W, True)
    W_kc = dense._WeightCache().get(W, False)
    outs = {"nt_fwd": empty_dense(T, C, dev), "nt_dP": empty_dense(T, K, dev)}
    calls = {"nt_fwd": lambda tile, o: dense.gemm_nt(P, W_ck, bias=b, out=o, math="bf16x6", tile=tile),
             "nt_dP": lambda tile, o: dense.gemm_nt(G, W_kc, out=o, math="bf16x6", tile=tile)}
    flops = {"nt_fwd": 2.0 * T * K * C, "nt_dP": 2.0 * T * C * K}
    tiles = [int(t) for t in a.tiles.split(",")]
    ref = {}
    for name, fn in calls.items():
        fn(0, outs[name])
        torch.cuda.synchronize()
        ref[name] = outs[name].clone()
    for r in range(a.rounds):
        for tile in tiles:
            rec = {"round": r, "tile": tile}
            for name, fn in calls.items():
                o = outs[name]
                for _ in range(3):
                    fn(tile, o)
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(a.reps):
                    fn(tile, o)
                e.record()
                torch.cuda.synchronize()
                ms = s.elapsed_time(e) / a.reps
                rec[name] = {"ms": round(ms, 4), "TFLOPs": round(flops[name] / (ms * 1e-3) / 1e12, 1),
                             "bitwise_tile0": bool(torch.equal(o, ref[name]))}
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
