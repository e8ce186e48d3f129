#!/usr/bin/env python
"""Fused output layer timing (Twitter-World 840k x 300 x 930 and Twitter-US 270k x 300 x 256),
every (math, tile) of gcg_project_softmax_xent, outputs checked against float64 on sampled rows.
`--bf16x6`: the bf16x6 tiles only; `--rounds R`: time every form R times, alternating."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphconvgeo_amd import dense  # noqa: E402
from graphconvgeo_amd.sparse import empty_dense  # noqa: E402
from oracle import gcn_oracle as O  # noqa: E402

BF_ONLY = "--bf16x6" in sys.argv
ROUNDS = int(sys.argv[sys.argv.index("--rounds") + 1]) if "--rounds" in sys.argv else 1
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
for T, K, C in ((840_000, 300, 930), (270_000, 300, 256)):
    P = empty_dense(T, K, dev).copy_(torch.randn((T, K), generator=g, device=dev) * 0.1)
    W = (torch.rand((K, C), generator=g, device=dev) * 2 - 1) * float(np.sqrt(6 / (K + C)))
    b = torch.randn(C, generator=g, device=dev) * 0.01
    y = torch.randint(0, C, (T,), generator=g, device=dev, dtype=torch.int32)
    Wp = dense._WeightCache().get(W, False)
    G = empty_dense(T, C, dev)
    loss = torch.empty(T, device=dev)
    hits = torch.empty(T, device=dev)
    torch.cuda.synchronize()
    rows = torch.randint(0, T, (400,), generator=g, device=dev)
    logits64 = P[rows].double() @ W.double() + b.double()
    _, l64, h64, G64 = O.softmax_xent_f64(logits64.cpu().numpy(), y[rows].cpu().numpy(), scale=1.0 / T)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    forms = [("bf16x6", t) for t in ((0, 1, 2, 3) if C > 768 else (0, 1, 3))]
    forms += [] if BF_ONLY else [("f32", t) for t in range(6)]
    for math, tile in [f for _ in range(ROUNDS) for f in forms]:
      f = lambda: dense._fused(P, Wp, b, y, 1.0 / T, None, G, loss, hits, math=math, tile=tile)  # noqa: E731
      f()
      torch.cuda.synchronize()
      err = max(float(np.abs(G[rows].cpu().numpy() - G64).max()) * T,
                float(np.abs(loss[rows].cpu().numpy() - l64).max()))
      res = []
      for _ in range(3):
        s.record()
        for _ in range(10):
            f()
        e.record()
        torch.cuda.synchronize()
        res.append(round(2.0 * T * K * C / (s.elapsed_time(e) / 10) / 1e9, 1))
      print(json.dumps({"shape": f"{T}x{K}x{C}", "math": math, "tile": tile, "TFLOPs": res, "max_err": err}),
            flush=True)
