"""Generate the committed golden fixtures (run in the build container, never on the GPU box).

python tests/golden/make_golden.py    ->  tests/golden/mention_graph.npz, geotext_synth.json

Pins the oracle against the reference itself where the reference is importable here:
  * The mention graph + projection come from the reference's own
    `data.DataLoader.get_graph` (data.py:302-375) and
    `efficient_collaboration_weighted_projected_graph2` (data.py:226-250), imported from
    /root/reference with three local shims (stub `haversine`, `builtins.xrange`,
    `np.Inf`). Theano/Lasagne/TensorFlow are not importable here, so the
    layer arithmetic is pinned against scipy (the executor of S.dot, scipy 1.15.3) and
    float64 numpy, evaluated exactly as tensormain.py / mlpconv.py spell it.
  * H is built with the literal tensormain.py:170-180 expression (modern-scipy fixes only:
    numpy for sp.sqrt/sp.isinf/sp.errstate, csr_matrix operands for `*`).
Only data (inputs and expected outputs) is written; no reference source is copied.
"""
from __future__ import annotations

import builtins
import hashlib
import json
import os
import sys
import types
import warnings

import numpy as np
import pandas as pd
import scipy.sparse as sps

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"


def import_reference_data_module():
    if REF not in sys.path:
        sys.path.insert(0, REF)
    h = types.ModuleType("haversine")
    h.haversine = lambda a, b: 0.0  # assignClasses only; unused by get_graph
    sys.modules.setdefault("haversine", h)
    builtins.xrange = range
    np.Inf = np.inf
    import data  # noqa: E402  (/root/reference/data.py)
    return data


def mention_tables(seed=77):
    """Synthetic train/dev/test user tables with @mentions (users, externals, celebrities)."""
    rng = np.random.default_rng(seed)
    names = [f"usr{chr(97 + i % 26)}{i:02d}" for i in range(64)]
    ext = [f"ext_{i:02d}" for i in range(24)]
    rows = []
    for i, u in enumerate(names):
        toks = ["hello", "world"]
        for m in rng.choice(len(names), size=rng.integers(0, 4), replace=False):
            toks.append("@" + names[m].upper() if rng.random() < 0.3 else "@" + names[m])
        for m in rng.choice(len(ext), size=rng.integers(0, 4), replace=False):
            toks.append("@" + ext[m])
        if i % 9 == 0:
            toks.append("@" + u)  # self-mention
        if i < 14:
            toks.append("@ext_hub")  # celebrity: degree > threshold -> removed
        rng.shuffle(toks)
        rows.append((u, 40.0 + rng.random(), -100.0 + rng.random(), " ".join(toks)))
    df = pd.DataFrame(rows, columns=["user", "lat", "lon", "text"]).set_index("user")
    df.sort_index(inplace=True)
    idx = rng.permutation(len(df))
    parts = [df.iloc[np.sort(idx[:40])], df.iloc[np.sort(idx[40:52])], df.iloc[np.sort(idx[52:])]]
    return [p.sort_index() for p in parts]


def literal_H(graph, n):
    """tensormain.py:170-180 (the float64 operator) with the modern-scipy fixes."""
    import networkx as nx

    adj = nx.adjacency_matrix(graph, nodelist=range(n), weight="w")
    adj = sps.csr_matrix(adj)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        adj.setdiag(1)
    n_, m = adj.shape
    diags = np.asarray(adj.sum(axis=1)).flatten()
    with np.errstate(divide="ignore"):
        diags_sqrt = 1.0 / np.sqrt(diags)
    diags_sqrt[np.isinf(diags_sqrt)] = 0
    D = sps.spdiags(diags_sqrt, [0], m, n_, format="csr")
    H = D * adj * D
    return adj, sps.csr_matrix(H.astype("float64"))


def relu(x):
    return x.dtype.type(0.5) * (x + np.abs(x))


def softmax(x):
    e = np.exp(x - x.max(axis=1, keepdims=True))
    return e / e.sum(axis=1, keepdims=True)


def make_mention_fixture():
    data = import_reference_data_module()
    dl = data.DataLoader(data_home="", celebrity_threshold=10)
    dl.df_train, dl.df_dev, dl.df_test = mention_tables()
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        dl.get_graph()
    g = dl.graph
    n = len(dl.df_train) + len(dl.df_dev) + len(dl.df_test)
    edges = np.array(sorted((min(a, b), max(a, b)) for a, b in g.edges()), dtype=np.int32)
    adj, H64_raw = literal_H(g, n)
    # main_mlpconv's H.astype('float32') (tensormain.py:221) canonicalizes the CSR (scipy's
    # astype sums duplicates and sorts indices), so the operator S.dot sees is sorted.
    H32 = H64_raw.astype(np.float32)
    assert H32.has_canonical_format
    H64 = H64_raw.copy()
    H64.sum_duplicates()
    rng = np.random.default_rng(7)
    K, F, C = 20, 30, 6
    Z = rng.standard_normal((n, K)).astype(np.float32)
    Y32 = np.asarray(H32 @ Z, dtype=np.float32)            # S.dot(H, Z) executor: scipy float32
    Y64 = H64 @ Z.astype(np.float64)
    # A 2-layer GCN forward (mlpconv.py:66-95) on a tiny BoW X, float32 and float64.
    X = sps.random(n, F, density=0.2, random_state=3, format="csr", dtype=np.float64)
    X.data += 0.05
    X = sps.csr_matrix(X.multiply(1.0 / np.maximum(np.sqrt(X.multiply(X).sum(axis=1)), 1e-12)))
    X = sps.csr_matrix(X, dtype=np.float32)
    X.sort_indices()
    W1 = rng.uniform(-0.4, 0.4, (F, K)).astype(np.float32)
    W2 = rng.uniform(-0.4, 0.4, (K, C)).astype(np.float32)
    b1 = rng.standard_normal(K).astype(np.float32) * 0.1
    b2 = rng.standard_normal(C).astype(np.float32) * 0.1
    idx = rng.integers(0, 40, size=30).astype(np.int32)  # train rows, with replacement
    y = rng.integers(0, C, size=30).astype(np.int32)
    Z1_32 = np.asarray(X @ W1, dtype=np.float32)
    h32 = relu(np.asarray(H32 @ Z1_32, dtype=np.float32) + b1)
    pre1_64 = H64 @ (sps.csr_matrix(X, dtype=np.float64) @ W1.astype(np.float64)) + b1
    h64 = relu(pre1_64)
    pre2_64 = H64 @ (h64 @ W2.astype(np.float64)) + b2
    P64 = softmax(pre2_64[idx])
    # float64 gradients of mean CE (no penalty) via the Theano rules.
    g_logits = P64.copy()
    g_logits[np.arange(idx.size), y] -= 1.0
    g_logits /= idx.size
    g_pre2 = np.zeros_like(pre2_64)
    np.add.at(g_pre2, idx, g_logits)
    g_Z2 = H64.T @ g_pre2
    g_W2 = h64.T @ g_Z2
    g_pre1 = (g_Z2 @ W2.astype(np.float64).T) * 0.5 * (1 + np.sign(pre1_64))
    g_W1 = sps.csr_matrix(X, dtype=np.float64).T @ (H64.T @ g_pre1)
    assert np.array_equal(H64.indices, H32.indices) and np.array_equal(H64.indptr, H32.indptr)
    out = dict(
        edges=edges, n=np.int64(n), adj_indptr=adj.indptr, adj_indices=adj.indices,
        H_indptr=H32.indptr.astype(np.int32), H_indices=H32.indices.astype(np.int32),
        H64_data=H64.data, H32_data=H32.data, H64_raw_sorted=np.bool_(H64_raw.has_sorted_indices), Z=Z, Y32=Y32, Y64=Y64,
        X_indptr=X.indptr, X_indices=X.indices, X_data=X.data, X_shape=np.array(X.shape),
        W1=W1, W2=W2, b1=b1, b2=b2, idx=idx, y=y, h32=h32, h64=h64, P64=P64,
        gW1_64=g_W1, gW2_64=g_W2, gb1_64=g_pre1.sum(0), gb2_64=g_pre2.sum(0),
    )
    np.savez_compressed(os.path.join(HERE, "mention_graph.npz"), **out)
    print(f"mention graph: {n} nodes, {len(edges)} edges, nnz(H)={H64.nnz}")


def sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def make_geotext_fixture():
    """Config 1/2: GEOTEXT-scale synthetic graph; pins the generator and scipy's H @ Z."""
    sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
    from graphconvgeo_amd.synth import synthetic_graph, dense

    H = synthetic_graph(9_475, 80_000)
    Z = dense(9_475, 300)
    Y = np.asarray(H @ Z, dtype=np.float32)  # scipy float32 = S.dot executor
    rec = {
        "n": 9475, "edges": 80000, "nnz": int(H.nnz), "K": 300,
        "sha256_indptr": sha(H.indptr.astype(np.int32)),
        "sha256_indices": sha(H.indices.astype(np.int32)),
        "sha256_data": sha(H.data.astype(np.float32)),
        "sha256_Z": sha(Z), "sha256_Y_scipy_f32": sha(Y),
        "sample_rows": [0, 1, 77, 4242, 9474],
        "Y_sample": Y[[0, 1, 77, 4242, 9474]].tolist(),
        "Y_rowsum_f64": float(Y.astype(np.float64).sum()),
    }
    with open(os.path.join(HERE, "geotext_synth.json"), "w") as f:
        json.dump(rec, f)
    print("geotext:", rec["nnz"], rec["sha256_Y_scipy_f32"][:16])


if __name__ == "__main__":
    make_mention_fixture()
    make_geotext_fixture()
