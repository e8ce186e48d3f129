#!/usr/bin/env python
"""The output layer (P.W2 + b2 -> softmax-CE, hits, dlogits; mlpconv.py:88-95) as one fused f32
MFMA launch (gcg_project_softmax_xent_weighted_f32) against the composition bf16x6 NT GEMM
(logits into G) + the row softmax-CE kernel in place (gcg_softmax_xent_weighted_f32): the
composition pays one more logits round trip through HBM and gains the bf16 matrix cores.
World (840k x 300 x 930) and Twitter-US (270k x 300 x 256) target shapes; HIP events, mean of
10, interleaved rounds; outputs compared (G max abs diff, loss / hits). Round 4, later: also the
fused layer on the bf16 matrix cores (gemm_fused6_kernel, GCG_FUSED_MATH=bf16x6)."""
import json
import math
import os
import sys

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
g = torch.Generator(device=dev).manual_seed(5)
for T, K, C in ((840_000, 300, 930), (270_000, 300, 256)):
    P = empty_dense(T, K, dev).copy_(torch.randn((T, K), generator=g, device=dev) * 0.1)
    W = (torch.rand((K, C), generator=g, device=dev) * 2 - 1) * math.sqrt(6.0 / (K + C))
    b = torch.randn(C, generator=g, device=dev) * 0.01
    y = torch.randint(0, C, (T,), generator=g, device=dev, dtype=torch.int32)
    Wp = dense._WeightCache().get(W, False)
    Wt = dense._WeightCache().get(W, True)
    G1, G2 = empty_dense(T, C, dev), empty_dense(T, C, dev)
    l1, l2 = torch.empty(T, device=dev), torch.empty(T, device=dev)
    h1, h2 = torch.empty(T, device=dev), torch.empty(T, device=dev)

    def fused():
        os.environ["GCG_FUSED_MATH"] = "f32"
        dense._fused(P, Wp, b, y, 1.0 / T, None, G1, l1, h1)

    def fused6():
        os.environ["GCG_FUSED_MATH"] = "bf16x6"
        os.environ.pop("GCG_FUSED6_WR", None)
        dense.FUSED_PRESPLIT = False
        dense._fused(P, Wp, b, y, 1.0 / T, None, G2, l2, h2)

    def fused6_wr2():
        os.environ["GCG_FUSED_MATH"] = "bf16x6"
        os.environ["GCG_FUSED6_WR"] = "2"
        dense.FUSED_PRESPLIT = False
        dense._fused(P, Wp, b, y, 1.0 / T, None, G2, l2, h2)
        os.environ.pop("GCG_FUSED6_WR", None)

    def fused6_fx():  # pre-split planes, the 32-row 4-wave tile
        os.environ["GCG_FUSED_MATH"] = "bf16x6"
        os.environ["GCG_FUSED6_FX_NARROW"] = "1"
        dense.FUSED_PRESPLIT = True
        dense._fused(P, Wp, b, y, 1.0 / T, None, G2, l2, h2)
        dense.FUSED_PRESPLIT = False
        os.environ.pop("GCG_FUSED6_FX_NARROW", None)

    def fused6_fx_wide():  # pre-split planes, the default tile (64 rows x 8 waves at N > 768)
        os.environ["GCG_FUSED_MATH"] = "bf16x6"
        dense.FUSED_PRESPLIT = True
        dense._fused(P, Wp, b, y, 1.0 / T, None, G2, l2, h2)
        dense.FUSED_PRESPLIT = False

    def fused6_wide():
        os.environ["GCG_FUSED_MATH"] = "bf16x6"
        os.environ["GCG_FUSED6_WIDE"] = "1"
        dense.FUSED_PRESPLIT = False
        dense._fused(P, Wp, b, y, 1.0 / T, None, G2, l2, h2)
        os.environ.pop("GCG_FUSED6_WIDE", None)

    def compose():
        dense.gemm_nt(P, Wt, bias=b, out=G2, math="bf16x6")
        dense._rows_call(G2, y, 1.0 / T, None, G2, l2, h2)

    fused()
    compose()
    torch.cuda.synchronize()
    rec = {"shape": f"{T}x{K}x{C}", "G_maxdiff": float((G1 - G2).abs().max()),
           "loss_maxdiff": float((l1 - l2).abs().max()), "hits_diff": float((h1 - h2).abs().sum())}
    fused6_fx()
    torch.cuda.synchronize()
    rec.update(G_maxdiff_presplit=float((G1 - G2).abs().max()),
               loss_maxdiff_presplit=float((l1 - l2).abs().max()),
               hits_diff_presplit=float((h1 - h2).abs().sum()))
    fused6_fx_wide()
    torch.cuda.synchronize()
    rec.update(G_maxdiff_presplit_wide=float((G1 - G2).abs().max()),
               loss_maxdiff_presplit_wide=float((l1 - l2).abs().max()),
               hits_diff_presplit_wide=float((h1 - h2).abs().sum()))
    fused6()
    torch.cuda.synchronize()
    rec.update(G_maxdiff_fused6=float((G1 - G2).abs().max()),
               loss_maxdiff_fused6=float((l1 - l2).abs().max()),
               hits_diff_fused6=float((h1 - h2).abs().sum()))
    flops = 2.0 * T * K * C
    for rnd in range(3):
        for name, fn in (("fused_f32", fused), ("compose_bf16x6", compose), ("fused_bf16x6", fused6),
                         ("fused_bf16x6_8waves", fused6_wr2), ("fused_bf16x6_wide", fused6_wide),
                         ("fused_bf16x6_presplit", fused6_fx), ("fused_bf16x6_presplit_wide", fused6_fx_wide)):
            ms = timeit(fn)
            rec.setdefault(name, []).append([round(ms, 3), round(flops / ms / 1e9, 1)])
    print(json.dumps(rec), flush=True)
    del P, G1, G2
    torch.cuda.empty_cache()
