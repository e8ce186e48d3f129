#!/usr/bin/env python
"""Timings of the dense output-layer products on one MI355X: the MFMA kernels of
csrc/dense.hip against torch (hipBLASLt GEMM + eager softmax/CE), HIP events, same stream.

Shapes (Twitter-World, SURVEY.md §8d: K = 300 hidden, C = 930 classes, T = 60 % of N rows):
  proj      logits = P . W2 + b2        T x 300 . 300 x 930   (propagate-first order)
  fused     loss, acc, (softmax-onehot)/T of P . W2 + b2  in one launch, vs
            torch addmm + log_softmax + nll + backward of the two (the logits gradient)
  dP        G . W2^T                   T x 930 . 930 x 300
  Z2        h . W2                     N x 300 . 300 x 930   (reference order)
  rows      softmax-CE of existing logits (reference order): loss pass + gradient pass, vs torch
FLOP = 2 M K N; the f32 MFMA dense peak is 157.3 TFLOP/s (MI355X_MICROARCH.md).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from graphconvgeo_amd import dense  # noqa: E402
from graphconvgeo_amd.sparse import empty_dense  # noqa: E402

PEAK_TF = 157.3


def time_op(fn, reps):
    fn()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(reps)]
    for a, b in evs:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in evs]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=840_000, help="T (target rows)")
    ap.add_argument("--nodes", type=int, default=1_400_000)
    ap.add_argument("--hidden", type=int, default=300)
    ap.add_argument("--classes", type=int, default=930)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--tiles", default="1,2,3,4,5", help="f32 fused-layer tiles to compare")
    ap.add_argument("--tn", default="1,2,3,6", help="gcg_gemm_tn tiles to compare")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    T, N, K, C = args.rows, args.nodes, args.hidden, args.classes
    g = torch.Generator(device=dev).manual_seed(0)
    P = empty_dense(T, K, dev).copy_(torch.randn((T, K), generator=g, device=dev) * 0.1)
    W = (torch.rand((K, C), generator=g, device=dev) * 2 - 1) * float(np.sqrt(6 / (K + C)))
    b = torch.zeros(C, device=dev)
    y = torch.randint(0, C, (T,), generator=g, device=dev)
    y32 = y.to(torch.int32)
    proj = dense.Projection()
    Wp = proj.fwd.get(W, False)
    Wt = proj.bwd.get(W, True)
    res = {}

    def rec(name, ms, flop=None, ref_ms=None):
        r = {"ms": round(ms, 4)}
        if flop:
            r["TFLOPs"] = round(flop / ms / 1e9, 1)
            r["frac_of_peak"] = round(flop / ms / 1e9 / PEAK_TF, 3)
        if ref_ms is not None:
            r["torch_ms"] = round(ref_ms, 4)
            if flop:
                r["torch_TFLOPs"] = round(flop / ref_ms / 1e9, 1)
            r["speedup"] = round(ref_ms / ms, 2)
        res[name] = r
        print(name, r, flush=True)

    out = empty_dense(T, C, dev)
    f = 2.0 * T * K * C
    G = empty_dense(T, C, dev)
    loss = torch.empty(T, device=dev)
    hits = torch.empty(T, device=dev)

    def ours_fused():
        dense._fused(P, Wp, b, y32, 1.0 / T, None, G, loss, hits)

    for tile in [int(t) for t in args.tiles.split(",") if t]:  # f32 fused tiles (B parts)
        rec(f"fused f32 tile {tile}",
            time_op(lambda: dense._fused(P, Wp, b, y32, 1.0 / T, None, G, loss, hits, math="f32",
                                         tile=tile), args.reps), f)
    rec("proj P.W2+b2", time_op(lambda: dense.gemm(P, Wp, bias=b, out=out), args.reps), f,
        time_op(lambda: torch.addmm(b, P, W), args.reps))

    def torch_fused():
        logits = torch.addmm(b, P, W)
        lp = torch.log_softmax(logits, dim=1)
        _l = -lp.gather(1, y.view(-1, 1)).mean()
        _acc = (logits.argmax(1) == y).float().mean()
        gl = torch.softmax(logits, dim=1)
        gl[torch.arange(T, device=dev), y] -= 1
        gl.mul_(1.0 / T)
        return gl

    rec("fused proj+softmax+CE+grad", time_op(ours_fused, args.reps), f,
        time_op(torch_fused, args.reps))
    Gc = G
    rec("dP = G.W2^T", time_op(lambda: dense.gemm(Gc, Wt), args.reps), f,
        time_op(lambda: torch.matmul(Gc, W.t()), args.reps))
    for tn in [int(t) for t in args.tn.split(",") if t]:  # split-K layouts (gcg_gemm_tn tiles)
        rec(f"dW2 = P^T.G tile={tn}", time_op(lambda: dense.gemm_tn(P, Gc, tile=tn), args.reps), f)
    rec("dW2 = P^T.G", time_op(lambda: dense.gemm_tn(P, Gc), args.reps), f,
        time_op(lambda: torch.matmul(P.t(), Gc), args.reps))
    del G, Gc, out
    h = empty_dense(N, K, dev).copy_(torch.rand((N, K), generator=g, device=dev))
    Z2 = empty_dense(N, C, dev)
    rec("Z2 = h.W2", time_op(lambda: dense.gemm(h, Wp, out=Z2), args.reps), 2.0 * N * K * C,
        time_op(lambda: torch.matmul(h, W), args.reps))
    rec("dW2 = h^T.dZ2 (reference order)", time_op(lambda: dense.gemm_tn(h, Z2), args.reps),
        2.0 * N * K * C, time_op(lambda: torch.matmul(h.t(), Z2), args.reps))
    del h, Z2
    logits = empty_dense(T, C, dev).copy_(torch.randn((T, C), generator=g, device=dev))
    gl = empty_dense(T, C, dev)
    one = torch.ones(1, device=dev)

    def ours_rows():
        dense._rows_call(logits, y32, 1.0, None, None, loss, hits)
        dense._rows_call(logits, y32, 1.0 / T, one, gl, loss, None)

    def torch_rows():
        lg = logits.detach().requires_grad_()
        lp = torch.log_softmax(lg, dim=1)
        l = -lp.gather(1, y.view(-1, 1)).mean()
        _acc = (lg.argmax(1) == y).float().mean()
        l.backward()
        return lg.grad

    rows_bytes = 3 * 4 * T * C  # read twice, write once
    ms = time_op(ours_rows, args.reps)
    rec("rows softmax-CE fwd+grad", ms, None, time_op(torch_rows, args.reps))
    res["rows softmax-CE fwd+grad"]["GBps"] = round(rows_bytes / ms / 1e6, 1)
    print(json.dumps({"shapes": {"T": T, "N": N, "K": K, "C": C}, "results": res}))


if __name__ == "__main__":
    main()
