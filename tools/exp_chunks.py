#!/usr/bin/env python
"""What the multi-GPU pipeline's split of one SpMM costs on one GPU.

World graph (power-law and uniform), K = 300, the bitwise mode 'auto' picks (ordered/rowwise):
  plain           one launch, full-width (1216-B) rows
  colchunks-c     the column-chunk pipeline's arithmetic: c launches over column slices
                  [c0, c1) of Z (views of the same stride-304 buffer, or separate chunk-wide
                  buffers as RowPartitionedCSR.spmm_pipelined allocates them)
  srcblocks-b     SURVEY.md §8e's source-block pipeline: H split into b column blocks (the
                  ranks' row ranges), one launch per block at full width, the first writing Y and
                  every later one continuing each row's storage-order sum from Y (accumulate)
  pipelined-c     RowPartitionedCSR.spmm_pipelined at world = 1 (includes its chunk copies)
HIP events, mean of 10 launches after 3 warm-ups."""
import os
import sys

import numpy as np
import scipy.sparse as sps
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphconvgeo_amd import sparse as gs  # noqa: E402
from graphconvgeo_amd.distributed import RowPartitionedCSR, row_partition  # noqa: E402
from graphconvgeo_amd.synth import CONFIGS, synthetic_graph  # noqa: E402

K = 300
dev = torch.device("cuda:0")
cfg = CONFIGS["twitter-world"]
kinds = (sys.argv[1] if len(sys.argv) > 1 else "powerlaw,uniform").split(",")


def timed(fn, reps=10):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


for kind in kinds:
    H = synthetic_graph(cfg.n_nodes, cfg.n_edges, kind=kind)
    n = H.shape[0]
    A = gs.DeviceCSR.from_scipy(H, dev, symmetric=True)
    mode = gs.resolve_auto(A)
    Z = gs.empty_dense(n, K, dev).copy_(torch.randn((n, K), device=dev))
    Y = gs.empty_dense(n, K, dev)
    ref = gs.spmm(A, Z, mode=mode).clone()
    res = {"plain": timed(lambda: gs.spmm(A, Z, out=Y, mode=mode))}
    for c in (2, 4):
        bounds = RowPartitionedCSR.chunk_bounds(K, c)
        res[f"colchunks-{c} (views)"] = timed(
            lambda: [gs.spmm(A, Z[:, a:b], out=Y[:, a:b], mode=mode) for a, b in bounds])
        assert torch.equal(Y, ref)
        bufs = [torch.empty((n, b - a), device=dev).copy_(Z[:, a:b]) for a, b in bounds]
        res[f"colchunks-{c} (chunk buffers)"] = timed(
            lambda: [gs.spmm(A, zb, out=Y[:, a:b], mode=mode) for zb, (a, b) in zip(bufs, bounds)])
        assert torch.equal(Y, ref)
        del bufs
    if hasattr(gs, "spmm_blocks"):
        for b in (2, 4, 8):
            blocks = gs.column_blocks(A, row_partition(H.indptr, b))
            res[f"srcblocks-{b}"] = timed(lambda: gs.spmm_blocks(blocks, Z, out=Y, mode=mode))
            assert torch.equal(Y, ref), "source-block accumulation is not bitwise"
            del blocks
    part = RowPartitionedCSR(H, 0, 1, dev, exchange="allgather")
    Zl = Z.contiguous()
    for c in (1, 2, 4):
        res[f"pipelined-{c}"] = timed(lambda: part.spmm_pipelined(Zl, Y, n_chunks=c, mode=mode))
    base = res["plain"]
    for name, ms in res.items():
        print(f"{kind} {mode} {name:28s} {ms:7.3f} ms  x{ms / base:.3f}", flush=True)
    del A, Z, Y, ref, part, Zl
    torch.cuda.empty_cache()
