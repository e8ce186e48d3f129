#!/usr/bin/env python
"""Child process of bench.py's live PMC pass (bench.py live_traffic): runs the bench's headline
SpMM launch -- the same graph (a .npz the parent wrote), the same empty_dense layout, mode and
gather hint -- under `rocprofv3 --pmc <counter>`, so the counters describe exactly the launch
the bench times. 1 plan-building call + `--warmup` untimed launches + `--launches` launches
timed back to back (wall clock, printed as a `PROBE {...}` line); the parent keeps only the
dispatches of the timed loop.

  rocprofv3 --pmc FETCH_SIZE -d DIR -o f -- python3 tools/pmc_probe.py GRAPH.npz --K 300 --mode ordered
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import scipy.sparse as sps
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphconvgeo_amd import sparse as gs  # noqa: E402
from graphconvgeo_amd.synth import SEED  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("graph")
    ap.add_argument("--K", type=int, default=300)
    ap.add_argument("--mode", default="auto")
    ap.add_argument("--launches", type=int, default=4)
    ap.add_argument("--warmup", type=int, default=0,
                    help="untimed launches after the plan-building one (the bench's --warmup)")
    a = ap.parse_args()
    with np.load(a.graph, allow_pickle=False) as f:
        n = int(f["n"])
        H = sps.csr_matrix((f["data"], f["indices"], f["indptr"]), shape=(n, n))
    dev = torch.device("cuda:0")
    A = gs.DeviceCSR.from_scipy(H, dev, symmetric=True)
    g = torch.Generator(device=dev).manual_seed(SEED)
    Z = gs.empty_dense(n, a.K, dev).copy_(torch.randn((n, a.K), generator=g, device=dev))
    Y = gs.empty_dense(n, a.K, dev)
    gs.spmm(A, Z, out=Y, mode=a.mode)  # plan + hint (dispatch dropped by the parent)
    for _ in range(a.warmup):  # dropped by the parent too
        gs.spmm(A, Z, out=Y, mode=a.mode)
    torch.cuda.synchronize()
    # the bench's timed loop: `launches` back-to-back launches between two synchronizations,
    # wall clock -- under the profiler, so the parent can state the profiler's own overhead
    t0 = time.perf_counter()
    for _ in range(a.launches):
        gs.spmm(A, Z, out=Y, mode=a.mode)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / max(a.launches, 1) * 1e3
    print("PROBE " + json.dumps({"n": n, "nnz": int(H.nnz), "K": a.K, "mode": a.mode,
                                 "warmup": a.warmup, "launches": a.launches,
                                 "ms_per_step": round(ms, 4)}), flush=True)


if __name__ == "__main__":
    main()
