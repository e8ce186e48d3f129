#!/usr/bin/env python
"""Split-K weight-gradient layouts (MG,NG,PD,WM,OCC[@slots]) INSIDE the training step (propagate-first order), where dW2
runs on a side stream beside the SpMM gathers: a one-wave-per-SIMD kernel cannot share a CU with
the gathers' waves, so standalone TFLOP/s do not rank the layouts there. GCG_TN variants (the
stacked X-head layout left alone: GCG_TN_NOT_STACKED=1), interleaved rounds, ms per step."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphconvgeo_amd.mlpconv import LasagneAdam, MLPCONV  # noqa: E402
from graphconvgeo_amd.synth import CONFIGS, synthetic_features, synthetic_graph  # noqa: E402

variants = os.environ.get("TN_INSTEP", "default;1,2,8,1;1,3,2,0,2;1,3,3,0,2;1,2,8,0,2;1,2,6,0,2").split(";")
orders = os.environ.get("TN_ORDERS", "propagate_first").split(",")
# TN_KNOB=GCG_TN_STACKED: vary the X-head gradient's layout (the stacked shapes) instead of dW2's
KNOB = os.environ.get("TN_KNOB", "GCG_TN")
os.environ["GCG_TN_NOT_STACKED"] = "1"
dev = torch.device("cuda:0")
for name, order in [(c, o) for c in (sys.argv[1] if len(sys.argv) > 1 else
                                     "twitter-us,twitter-world").split(",") for o in orders]:
    cfg = CONFIGS[name]
    H = synthetic_graph(cfg.n_nodes, cfg.n_edges)
    X = synthetic_features(cfg.n_nodes, cfg.n_features, nnz_per_row=64)
    n = cfg.n_nodes
    rng = np.random.default_rng(77)
    Y = rng.integers(0, cfg.n_classes, size=n)
    Y[:cfg.n_classes] = np.arange(cfg.n_classes)
    n_tr = int(0.6 * n)
    train = rng.choice(n_tr, size=n_tr).astype(np.int32)
    clf = MLPCONV(n_epochs=0, hidden_layer_size=cfg.hidden, device=dev, seed=1,
                  order=order)
    clf.fit(X, train, np.arange(n_tr, int(0.8 * n), dtype=np.int32),
            np.arange(int(0.8 * n), n, dtype=np.int32), Y, H)
    y_train = torch.as_tensor(Y[train].astype(np.int32), device=dev)
    opt = LasagneAdam(clf.params)
    clf.n_epochs = 1
    step0 = clf._make_train_step(opt, y_train)
    # TN_MAIN_PRIO=1: the step on a high-priority stream (the weight-gradient side stream keeps
    # the default priority), so the dispatcher prefers the critical path's workgroups
    hi = torch.cuda.Stream(device=dev, priority=-1) if os.environ.get("TN_MAIN_PRIO") == "1" else None

    def step():
        if hi is None:
            return step0()
        hi.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(hi):
            step0()
        torch.cuda.current_stream(dev).wait_stream(hi)
    res = {}
    for rnd in range(3):
        for v in variants:
            os.environ.pop(KNOB, None)
            os.environ.pop("GCG_TN_SLOTS", None)
            if v != "default":
                tile, _, slots = v.partition("@")
                os.environ[KNOB] = tile
                if slots:
                    os.environ["GCG_TN_SLOTS"] = slots
            for _ in range(2):
                step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(5):
                step()
            torch.cuda.synchronize()
            res.setdefault(v, []).append(round((time.perf_counter() - t0) / 5 * 1e3, 3))
    os.environ.pop(KNOB, None)
    os.environ.pop("GCG_TN_SLOTS", None)
    print(json.dumps({"config": name, "order": order, "main_prio": hi is not None,
                      "ms_per_step": res}), flush=True)
    del clf, step, opt
    torch.cuda.empty_cache()
