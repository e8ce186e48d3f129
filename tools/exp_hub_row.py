#!/usr/bin/env python
"""Time of hub rows alone (ordered mode): R rows of L nonzeros each gathering random rows of a
Twitter-World-sized Z (1.4M x 300), single-wave (GCG_COOP_MIN=-1) vs whole-workgroup rows.
HIP events, mean of 10 after 3 warm-ups."""
import os
import sys

import numpy as np
import scipy.sparse as sps
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphconvgeo_amd import sparse as gs  # noqa: E402

dev = torch.device("cuda:0")
N, K = 1_400_000, 300
Z = gs.empty_dense(N, K, dev).normal_()
rng = np.random.default_rng(0)
for R, L in ((1, 12189), (1, 4096), (1, 1024), (64, 12189), (256, 12189), (1024, 2048)):
    idx = np.sort(rng.integers(0, N, size=(R, L)), axis=1).astype(np.int32).ravel()
    H = sps.csr_matrix((np.full(R * L, 0.01, np.float32), idx, np.arange(0, R * L + 1, L)),
                       shape=(R, N))
    A = gs.DeviceCSR.from_scipy(H, dev)
    Y = gs.empty_dense(R, K, dev)
    f = lambda: gs.spmm(A, Z, out=Y, mode="ordered", task_nnz=512)
    for _ in range(3):
        f()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(10):
        f()
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / 10
    print(f"coop_min={os.environ.get('GCG_COOP_MIN', 'default')} rows={R} nnz/row={L} "
          f"ms={ms:.3f} GB/s={R * L * 1216 / ms / 1e6:.1f}", flush=True)
