#!/usr/bin/env python
"""Row-partitioned GCN training step (graphconvgeo_amd.dist_train) on N GPUs of one node.

  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \\
      tools/bench_train_dist.py --config twitter-world [--order propagate_first]

One step = fwd + bwd + one bucketed gradient all-reduce + Lasagne Adam, the whole synthetic
graph (same data as tools/bench_train.py, seed 77) split by rows over the ranks. Timing: W
untimed steps, barrier + synchronize, K timed steps, barrier + synchronize, max over ranks.
`--dist-backend gloo` rehearses several ranks on one GPU (not a performance number).
`--phases` (round 4): one step is recorded (distributed.TRACE) and its exchanges and local
SpMMs are replayed alone, so the line shows how much of the exchange the pipelined step hides:
exchange_alone + spmm_alone against the step, and the step with the pipeline switched off
(--chunks 1 on every propagate) beside it.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from graphconvgeo_amd.dist_train import RowPartitionedGCN  # noqa: E402
from graphconvgeo_amd.synth import CONFIGS, synthetic_features, synthetic_graph  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="twitter-us", choices=sorted(CONFIGS))
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--nnz-per-row", type=int, default=64)
    ap.add_argument("--order", default="propagate_first", choices=["reference", "propagate_first"])
    ap.add_argument("--exchange", default="auto", choices=["auto", "allgather", "mesh", "halo"])
    ap.add_argument("--chunks", type=int, default=0, help="column chunks (0 = auto)")
    ap.add_argument("--phases", action="store_true",
                    help="replay one step's exchanges and local SpMMs alone; time --chunks 1")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"])
    args = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dev_index = local_rank % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    if world > 1:
        from graphconvgeo_amd.distributed import init_process_group
        init_process_group(args.dist_backend, dev if args.dist_backend == "nccl" else None)
    cfg = CONFIGS[args.config]
    t0 = time.perf_counter()
    H = synthetic_graph(cfg.n_nodes, cfg.n_edges)
    X = synthetic_features(cfg.n_nodes, cfg.n_features, nnz_per_row=args.nnz_per_row)
    n = cfg.n_nodes
    rng = np.random.default_rng(77)
    Y = rng.integers(0, cfg.n_classes, size=n)
    Y[:cfg.n_classes] = np.arange(cfg.n_classes)
    n_tr = int(0.6 * n)
    train = rng.choice(n_tr, size=n_tr).astype(np.int32)
    t_gen = time.perf_counter() - t0
    model = RowPartitionedGCN(H, X, train, Y, cfg.hidden, cfg.n_classes, rank, world, dev,
                              order=args.order, exchange=args.exchange)
    model.part.chunks_override = args.chunks or None
    opt = model.make_optimizer()

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)

    def timed(fn, reps):
        barrier()
        t0 = time.perf_counter()
        out = None
        for _ in range(reps):
            out = fn()
        barrier()
        el = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([el], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el / max(reps, 1) * 1e3, out

    for _ in range(args.warmup):
        model.train_step(opt)
    ms, (loss, acc) = timed(lambda: model.train_step(opt), args.steps)
    phases = None
    if args.phases:
        from graphconvgeo_amd import distributed as D
        D.TRACE = []
        model.train_step(opt)
        rec, D.TRACE = D.TRACE, None

        def exchanges():
            for _f, _A, bufs, _o, _b, _g, _kw in rec:
                for _c0, _c1, buf in bufs.chunks:
                    D._wait(bufs.layout.exchange(buf, async_op=False))

        def spmms():
            for f, A, bufs, out, bias, gate, kw in rec:
                for c0, c1, buf in bufs.chunks:
                    f(A, buf[:, :c1 - c0], out[:, c0:c1], bias=None if bias is None else bias[c0:c1],
                      gate=None if gate is None else gate[:, c0:c1], **kw)
        reps = max(args.steps // 2, 2)
        t_x, _ = timed(exchanges, reps)
        t_s, _ = timed(spmms, reps)
        model.part.chunks_override = 1
        for _ in range(2):
            model.train_step(opt)
        t_1, _ = timed(lambda: model.train_step(opt), reps)
        model.part.chunks_override = args.chunks or None
        phases = {"propagates_per_step": len(rec),
                  "chunks": [len(b.chunks) for _f, _A, b, *_r in rec],
                  "exchange_bytes_in_rank0": sum(b.layout.bytes_in(o.shape[1]) for _f, _A, b, o, *_r in rec),
                  "exchange_alone_ms": round(t_x, 3), "local_spmm_alone_ms": round(t_s, 3),
                  "step_ms": round(ms, 3), "step_unpipelined_ms": round(t_1, 3),
                  "hidden_ms": round(t_1 - ms, 3)}
    if rank == 0:
        print(json.dumps({
            "metric": "row-partitioned GCN fwd+bwd+allreduce+adam step", "config": cfg.name,
            "n_gpus": world, "ms_per_step": round(ms, 3), "order": args.order,
            "exchange": model.part.exchange, "halo_fraction": round(model.part.halo_fraction, 4),
            "rows_rank0": model.part.n_local, "targets_total": model.T_total,
            "loss": float(loss), "acc": float(acc), "backend": args.dist_backend if world > 1 else None,
            "data_gen_s": round(t_gen, 1), "phases": phases}), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
