#!/usr/bin/env python
"""X.W1 (mlpconv.py:71, the K2 product of the sparse-input layer) as one storage-order gather
vs split like DeviceCSR.tmatmul: X's dense Zipf-head columns (sparse._dense_column_split) as a
dense N x Fh block times W1's head rows on the bf16x6 MFMA GEMM, the rest a CSR gather, then
the two added. HIP events, mean of `reps` after warm-up; prints one JSON line per config
with each part's time and the max deviation from the gather (not bitwise: a different
summation order).

  python tools/exp_xw_split.py --config twitter-world
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphconvgeo_amd import dense  # noqa: E402
from graphconvgeo_amd import sparse as gs  # noqa: E402
from graphconvgeo_amd.synth import CONFIGS, synthetic_features  # noqa: E402


def timeit(fn, reps):
    for _ in range(2):
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
    ap.add_argument("--config", default="twitter-world", choices=sorted(CONFIGS))
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    cfg = CONFIGS[a.config]
    dev = torch.device("cuda:0")
    X = synthetic_features(cfg.n_nodes, cfg.n_features)
    Xd = gs.DeviceCSR.from_scipy(X, dev)
    K = cfg.hidden
    g = torch.Generator(device=dev).manual_seed(3)
    W1 = torch.randn((cfg.n_features, K), generator=g, device=dev) * 0.05
    n = X.shape[0]
    Z = gs.empty_dense(n, K, dev)
    rec = {"config": a.config, "N": n, "F": cfg.n_features, "K": K, "nnz_X": int(X.nnz)}
    rec["gather_ms"] = round(timeit(lambda: gs.spmm(Xd, W1, out=Z), a.reps), 3)
    Zref = Z.clone()
    cand, Xh, tail_t = Xd._dense_column_split()
    tail = tail_t.transpose()
    rec["head_cols"] = int(cand.numel())
    rec["tail_nnz"] = int(tail.nnz)
    Zt = gs.empty_dense(n, K, dev)
    Zh = gs.empty_dense(n, K, dev)
    Wh_t = W1.index_select(0, cand).t().contiguous()  # K x Fh: the NT GEMM's Bt
    rec["tail_gather_ms"] = round(timeit(lambda: gs.spmm(tail, W1, out=Zt), a.reps), 3)
    for math in ("bf16x6", "f32"):
        rec[f"head_gemm_{math}_ms"] = round(timeit(
            lambda: dense.gemm_nt(Xh, Wh_t, out=Zh, math=math), a.reps), 3)
    rec["add_ms"] = round(timeit(lambda: torch.add(Zt, Zh, out=Z), a.reps), 3)
    side = torch.cuda.Stream(dev)

    def split():
        main = torch.cuda.current_stream(dev)
        side.wait_stream(main)
        with torch.cuda.stream(side):
            dense.gemm_nt(Xh, Wh_t, out=Zh, math="bf16x6")
        gs.spmm(tail, W1, out=Zt)
        main.wait_stream(side)
        torch.add(Zt, Zh, out=Z)
    rec["split_total_ms"] = round(timeit(split, a.reps), 3)
    d = (Z - Zref).abs().max().item()
    rec["max_abs_dev"] = d
    rec["max_rel_dev"] = d / max(Zref.abs().max().item(), 1e-30)
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
