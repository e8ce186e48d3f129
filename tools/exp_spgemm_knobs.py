"""Experiment: SpGEMM launch knobs at Twitter-World (side stream, small-row grid)."""
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
for side in ["0"]:
    for grid in ["0", "4096"]:
        os.environ["GCG_SPGEMM_NO_SIDE"] = "0" if side == "1" else "1"
        os.environ["GCG_SPGEMM_SMALL_GRID"] = grid
        ts = []
        for _ in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            C = gs.spgemm(H, X)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
            del C
        print(f"side={side} small_grid={grid} ms={1e3 * np.median(ts):.1f}", flush=True)
