#!/usr/bin/env python
"""Library A/B of the SpMM side: the bench's headline launch (World power-law H.Z, K = 300,
auto mode, empty_dense layout, HIP events, mean of 20 after 5) and the Twitter-US training
step in MLPCONV's default order (wall clock, 10 steps after 5). One process per library
(GCG_LIB), alternated `--rounds=` times; one JSON line per (round, library).

  python tools/exp_step_ab.py tools/varlibs/libgcg_a.so graphconvgeo_amd/libgcg_spmm.so
"""
import json
import os
import subprocess
import sys

CHILD = r'''
import json, os, sys, time, numpy as np, torch
sys.path.insert(0, os.getcwd())
from graphconvgeo_amd import sparse as gs
from graphconvgeo_amd.synth import CONFIGS, SEED, synthetic_graph, synthetic_features
from graphconvgeo_amd.mlpconv import MLPCONV, LasagneAdam
dev = torch.device("cuda:0")
out = {}
cfg = CONFIGS["twitter-world"]
H = synthetic_graph(cfg.n_nodes, cfg.n_edges)
A = gs.DeviceCSR.from_scipy(H, dev)
g = torch.Generator(device=dev).manual_seed(SEED)
Z = gs.empty_dense(H.shape[0], 300, dev).copy_(torch.randn((H.shape[0], 300), generator=g, device=dev))
Y = gs.empty_dense(H.shape[0], 300, dev)
for _ in range(5): gs.spmm(A, Z, out=Y)
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(20): gs.spmm(A, Z, out=Y)
e.record(); torch.cuda.synchronize()
out["headline_ms"] = round(s.elapsed_time(e) / 20, 4)
del A, Z, Y, H
cfg = CONFIGS["twitter-us"]
H = synthetic_graph(cfg.n_nodes, cfg.n_edges)
X = synthetic_features(cfg.n_nodes, cfg.n_features, nnz_per_row=64)
n = cfg.n_nodes
rng = np.random.default_rng(SEED)
Yl = rng.integers(0, cfg.n_classes, size=n)
n_tr = int(0.6 * n)
train = rng.choice(n_tr, size=n_tr).astype(np.int32)
clf = MLPCONV(n_epochs=0, hidden_layer_size=cfg.hidden, device=dev, seed=1)
clf.fit(X, train, np.arange(n_tr, int(0.8 * n), dtype=np.int32), np.arange(int(0.8 * n), n, dtype=np.int32), Yl, H)
step = clf._make_train_step(LasagneAdam(clf.params), torch.as_tensor(Yl[train].astype(np.int32), device=dev))
for _ in range(5): step()
torch.cuda.synchronize(); t0 = time.perf_counter()
for _ in range(10): step()
torch.cuda.synchronize()
out["us_step_ms"] = round((time.perf_counter() - t0) / 10 * 1e3, 3)
out["order"] = clf.l_out.order
print("R " + json.dumps(out), flush=True)
'''


def main():
    libs = [a for a in sys.argv[1:] if not a.startswith("--")]
    rounds = 2
    for a in sys.argv[1:]:
        if a.startswith("--rounds="):
            rounds = int(a.split("=")[1])
    for r in range(rounds):
        for lib in libs:
            env = dict(os.environ, GCG_LIB=os.path.abspath(lib))
            p = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True,
                               timeout=400)
            line = next((ln for ln in p.stdout.splitlines() if ln.startswith("R ")), None)
            rec = {"round": r, "lib": lib}
            rec.update(json.loads(line[2:]) if line else {"error": (p.stderr or p.stdout)[-400:]})
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
