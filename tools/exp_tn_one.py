#!/usr/bin/env python
"""Split-K weight-gradient GEMM C = A^T.B timing at the training step's shapes: XCD-aware tile
order off / on (GCG_TN_XCD, outputs compared bitwise) and tile variants (GCG_TN=MG,NG,PD)."""
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
          (1_400_000, 256, 300, "World X-head^T.dZ1")]
for R, M, N, what in shapes:
    A = empty_dense(R, M, dev).copy_(torch.randn((R, M), generator=g, device=dev))
    B = empty_dense(R, N, dev).copy_(torch.randn((R, N), generator=g, device=dev))
    outs, res = {}, {}
    for xcd in ("0", "1", "1,1,8", "1,1,16", "1,2,4"):
        os.environ["GCG_TN_XCD"] = xcd[0]
        if "," in xcd:
            os.environ["GCG_TN"] = xcd
        else:
            os.environ.pop("GCG_TN", None)
        outs[xcd] = dense.gemm_tn(A, B).clone()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        r = []
        for _ in range(3):
            s.record()
            for _ in range(5):
                dense.gemm_tn(A, B)
            e.record()
            torch.cuda.synchronize()
            r.append(round(2.0 * R * M * N / (s.elapsed_time(e) / 5) / 1e9, 1))
        res[xcd] = r
    os.environ.pop("GCG_TN", None)
    print(json.dumps({"shape": f"{R}x{M}x{N}", "what": what, "TFLOPs": res,
                      "bitwise_xcd": bool(torch.equal(outs["0"], outs["1"]))}), flush=True)
    del A, B
