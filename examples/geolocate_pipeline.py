#!/usr/bin/env python
"""End-to-end GCN geolocation on synthetic tweets, following tensormain.py's pipeline with
the graph work and the training on the GPU:

  host  (as data.py)      user tables -> @mention incidences, TF-IDF features, region labels
  GPU   gcg_project_mention_graph    celebrity filter + projection  (data.py:226-250,364-373)
  GPU   gcg_normalize_adjacency_f32  H = D^-1/2 (A+I) D^-1/2          (tensormain.py:168-181)
  GPU   MLPCONV.fit / accuracy / predict                              (tensormain.py:207-244)

Synthetic data: users live in one of `regions`; they mention other users mostly from their
own region and use region-specific words, so the graph and the text both carry the label.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import pandas as pd

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def synthetic_tables(n_users=6000, regions=12, seed=77):
    rng = np.random.default_rng(seed)
    names = np.array([f"user{i:05d}" for i in range(n_users)])
    region = rng.integers(0, regions, n_users)
    words = [[f"w{r}x{j}" for j in range(40)] for r in range(regions)]
    common = [f"common{j}" for j in range(200)]
    by_region = [np.flatnonzero(region == r) for r in range(regions)]
    rows = []
    for i in range(n_users):
        r = region[i]
        toks = list(rng.choice(words[r], 8)) + list(rng.choice(common, 12))
        for _ in range(rng.integers(0, 5)):
            pool = by_region[r] if rng.random() < 0.8 else np.arange(n_users)
            toks.append("@" + names[rng.choice(pool)])
        for _ in range(rng.integers(0, 3)):
            toks.append(f"@ext{r}_{rng.integers(0, 30)}")  # shared external handles
        rng.shuffle(toks)
        rows.append((names[i], 40.0 + r + rng.random(), -100.0 + rng.random(), " ".join(toks)))
    df = pd.DataFrame(rows, columns=["user", "lat", "lon", "text"]).set_index("user").sort_index()
    perm = rng.permutation(n_users)
    n_tr, n_dev = int(0.7 * n_users), int(0.15 * n_users)
    parts = [df.iloc[np.sort(perm[:n_tr])], df.iloc[np.sort(perm[n_tr:n_tr + n_dev])],
             df.iloc[np.sort(perm[n_tr + n_dev:])]]
    return [p.sort_index() for p in parts], regions


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--users", type=int, default=6000)
    ap.add_argument("--epochs", type=int, default=100)
    ap.add_argument("--hidden", type=int, default=64)
    ap.add_argument("--celebrity", type=int, default=10)
    args = ap.parse_args()
    import scipy.sparse as sps
    import torch
    from sklearn.feature_extraction.text import TfidfVectorizer

    from graphconvgeo_amd.mentions import mention_graph_operator
    from graphconvgeo_amd.mlpconv import MLPCONV

    (df_train, df_dev, df_test), regions = synthetic_tables(args.users)
    t0 = time.perf_counter()
    H = mention_graph_operator(df_train, df_dev, df_test, celebrity_threshold=args.celebrity,
                               device="cuda")
    t_graph = time.perf_counter() - t0
    # data.py:378-397 (token pattern drops @mentions; binary tf, l2 norm)
    vec = TfidfVectorizer(token_pattern=r"(?u)(?<![#@])\b\w\w+\b", binary=True, norm="l2",
                          min_df=2, max_df=0.5, dtype=np.float32)
    X = sps.vstack([vec.fit_transform(df_train.text.values), vec.transform(df_dev.text.values),
                    vec.transform(df_test.text.values)]).tocsr().astype(np.float32)
    lab = lambda df: (df["lat"].values - 40.0).astype(int)  # region labels (stand-in for kdtree)
    Y = np.concatenate([lab(df_train), lab(df_dev), lab(df_test)])
    n_tr, n_dev = len(df_train), len(df_dev)
    train = np.random.default_rng(77).choice(n_tr, size=n_tr).astype(np.int32)  # tensormain.py:226
    dev = np.arange(n_tr, n_tr + n_dev, dtype=np.int32)
    test = np.arange(n_tr + n_dev, len(Y), dtype=np.int32)
    clf = MLPCONV(n_epochs=args.epochs, hidden_layer_size=args.hidden, regul_coefs=[1e-6, 1e-6],
                  early_stopping_max_down=5, dtype="float32", use_graph=True)
    t0 = time.perf_counter()
    clf.fit(X, train, dev, test, Y, H)
    torch.cuda.synchronize()
    t_fit = time.perf_counter() - t0
    acc = clf.accuracy("test", Y[test])
    print(json.dumps({"users": len(Y), "graph_nnz": H.nnz, "features": X.shape[1],
                      "graph_build_s": round(t_graph, 3), "fit_s": round(t_fit, 3),
                      "epochs_run": len(clf.history), "test_acc": round(acc, 4),
                      "chance": round(1.0 / regions, 4)}))
    return acc


if __name__ == "__main__":
    main()
