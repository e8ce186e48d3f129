"""Experiment: where the Twitter-World SpGEMM wall time goes outside its kernels.

Times gs.spgemm per call (a) dropping the previous result first, (b) keeping it alive (as
tools/bench_graph.py does), (c) the bare torch.empty of the products-sized output, and (d)
(a) again with the HIP default mempool's release threshold raised, so the library's
stream-ordered temporaries stay mapped between calls.
"""
import ctypes
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphconvgeo_amd import sparse as gs  # noqa: E402
from graphconvgeo_amd.synth import CONFIGS, synthetic_graph, synthetic_features  # noqa: E402

cfg = CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "twitter-world"]
dev = torch.device("cuda")
H = gs.DeviceCSR.from_scipy(synthetic_graph(cfg.n_nodes, cfg.n_edges), dev)
X = gs.DeviceCSR.from_scipy(synthetic_features(cfg.n_nodes, cfg.n_features), dev)
P = int(np.diff(X.indptr.cpu().numpy())[H.indices.cpu().numpy()].sum())


def wall(fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = fn()
    torch.cuda.synchronize()
    return r, (time.perf_counter() - t0) * 1e3


def report(tag, ts):
    print(f"{tag}: " + " ".join(f"{t:.1f}" for t in ts) + f" ms  reserved={torch.cuda.memory_reserved() / 2**30:.1f} GiB",
          flush=True)


ts = []
for _ in range(4):
    C, t = wall(lambda: gs.spgemm(H, X))
    ts.append(t)
    del C
report("drop previous", ts)

ts, keep = [], None
for _ in range(4):
    keep, t = wall(lambda: gs.spgemm(H, X))
    ts.append(t)
report("keep previous", ts)
del keep

ts, keep = [], None
for _ in range(4):
    keep, t = wall(lambda: (torch.empty(P, dtype=torch.int32, device=dev),
                            torch.empty(P, dtype=torch.float32, device=dev)))
    ts.append(t)
report("torch.empty(P) x2, keep previous", ts)
del keep

hip = ctypes.CDLL("libamdhip64.so")
pool = ctypes.c_void_p()
assert hip.hipDeviceGetDefaultMemPool(ctypes.byref(pool), 0) == 0
thr = ctypes.c_uint64(2**64 - 1)
assert hip.hipMemPoolSetAttribute(pool, 4, ctypes.byref(thr)) == 0  # hipMemPoolAttrReleaseThreshold
ts = []
for _ in range(4):
    C, t = wall(lambda: gs.spgemm(H, X))
    ts.append(t)
    del C
report("drop previous, mempool keeps temporaries", ts)
