"""CPU tests: the oracle against the golden fixtures and against scipy (the S.dot executor).

These pin the checker before any GPU result is compared with it.
"""
import json
import os

import networkx as nx
import numpy as np
import pytest
import scipy.sparse as sps

from graphconvgeo_amd.graph import csr_from_edges, normalize_adjacency
from graphconvgeo_amd.synth import dense, synthetic_graph
from oracle import gcn_oracle as O

GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def mention():
    return dict(np.load(os.path.join(GOLD, "mention_graph.npz")))


def _H(g, dtype="H32_data"):
    n = int(g["n"])
    return sps.csr_matrix((g[dtype].copy(), g["H_indices"].copy(), g["H_indptr"].copy()),
                          shape=(n, n))


def test_normalization_matches_reference_expression(mention):
    """Oracle + product H construction == tensormain.py:170-180 run by the fixture script."""
    n = int(mention["n"])
    adj = sps.csr_matrix((np.ones(mention["adj_indices"].size), mention["adj_indices"],
                          mention["adj_indptr"]), shape=(n, n))
    H_or = O.normalize_adjacency(adj, out_dtype=np.float64)
    H_ref = _H(mention, "H64_data")
    H_ref.sort_indices()
    assert np.array_equal(H_or.indptr, H_ref.indptr)
    assert np.array_equal(H_or.indices, H_ref.indices)
    assert np.array_equal(H_or.data, H_ref.data)  # bitwise float64
    # product-side builders agree too
    u, v = mention["edges"][:, 0], mention["edges"][:, 1]
    H_e = csr_from_edges(n, u, v, dtype=np.float64)
    assert np.array_equal(H_e.data, H_ref.data) and np.array_equal(H_e.indices, H_ref.indices)
    g = nx.Graph()
    g.add_nodes_from(range(n))
    g.add_edges_from(mention["edges"].tolist())
    H_p = normalize_adjacency(g, n, dtype=np.float64)
    H_p.sort_indices()
    assert np.array_equal(H_p.data, H_ref.data)


def test_H_properties(mention):
    H = _H(mention, "H64_data")
    assert (abs(H - H.T) > 0).nnz == 0  # symmetric -> H^T = H in backward
    assert H.nnz == 2 * len(mention["edges"]) + int(mention["n"])
    assert np.all(H.diagonal() > 0)


def test_spmm_oracle_bitwise_vs_golden(mention):
    H = _H(mention)
    assert np.array_equal(O.spmm_f32(H, mention["Z"]), mention["Y32"])
    assert np.abs(O.spmm_f64(_H(mention, "H64_data"), mention["Z"]) - mention["Y64"]).max() < 1e-12


def test_gcn_forward_backward_vs_golden(mention):
    n = int(mention["n"])
    X = sps.csr_matrix((mention["X_data"], mention["X_indices"], mention["X_indptr"]),
                       shape=tuple(mention["X_shape"]))
    H = _H(mention)
    g = mention
    f32 = O.gcn_forward(X, H, g["W1"], g["b1"], g["W2"], g["b2"], g["idx"], dtype=np.float32)
    assert np.array_equal(f32["h"], g["h32"])  # scipy-order fp32, bitwise
    f64 = O.gcn_forward(X, _H(g, "H64_data"), g["W1"], g["b1"], g["W2"], g["b2"], g["idx"])
    assert np.abs(f64["h"] - g["h64"]).max() < 1e-12
    assert np.abs(f64["P"] - g["P64"]).max() < 1e-12
    assert np.abs(f32["P"] - g["P64"]).max() < 1e-5
    gr = O.gcn_backward(X, _H(g, "H64_data"), g["W1"], g["W2"], f64, g["idx"], g["y"], (0.0, 0.0))
    for k in ("W1", "W2", "b1", "b2"):
        assert np.abs(gr[k] - g[f"g{k}_64"]).max() < 1e-12, k
    assert n == H.shape[0]


def test_gradients_by_finite_differences(mention):
    """The Theano-rule backward (incl. L1/L2 shares) equals a numerical derivative."""
    g = mention
    X = sps.csr_matrix((g["X_data"], g["X_indices"], g["X_indptr"]), shape=tuple(g["X_shape"]))
    H = _H(g, "H64_data")
    W1 = g["W1"].astype(np.float64)
    W2 = g["W2"].astype(np.float64)
    coefs = (1e-3, 2e-3)

    def loss(W1_, W2_):
        f = O.gcn_forward(X, H, W1_, g["b1"], W2_, g["b2"], g["idx"])
        return O.gcn_loss(f["P"], g["y"], W1_, W2_, coefs)

    f = O.gcn_forward(X, H, W1, g["b1"], W2, g["b2"], g["idx"])
    gr = O.gcn_backward(X, H, W1, W2, f, g["idx"], g["y"], coefs)
    eps = 1e-6
    for (i, j) in [(0, 0), (3, 5), (7, 2)]:
        Wp = W2.copy(); Wp[i, j] += eps
        Wm = W2.copy(); Wm[i, j] -= eps
        num = (loss(W1, Wp) - loss(W1, Wm)) / (2 * eps)
        assert abs(num - gr["W2"][i, j]) < 1e-6
        Wp = W1.copy(); Wp[i, j] += eps
        Wm = W1.copy(); Wm[i, j] -= eps
        num = (loss(Wp, W2) - loss(Wm, W2)) / (2 * eps)
        assert abs(num - gr["W1"][i, j]) < 1e-6


def test_oracle_equals_scipy_on_unsorted_and_duplicate_csr():
    rng = np.random.default_rng(0)
    n, m, nnz = 300, 200, 4000
    rows = np.sort(rng.integers(0, n, nnz))
    cols = rng.integers(0, m, nnz)
    indptr = np.searchsorted(rows, np.arange(n + 1)).astype(np.int32)
    H = sps.csr_matrix((rng.standard_normal(nnz).astype(np.float32), cols.astype(np.int32), indptr),
                       shape=(n, m))
    assert not H.has_canonical_format
    Z = rng.standard_normal((m, 37)).astype(np.float32)
    assert np.array_equal(O.spmm_f32(H, Z), H @ Z)
    b = rng.standard_normal(37).astype(np.float32)
    r = rng.integers(0, n, 50)
    ref = (H @ Z + b)[r]
    assert np.array_equal(O.spmm_f32(H, Z, bias=b, act="relu", rows=r), 0.5 * (ref + np.abs(ref)))


def test_geotext_fixture_pins_generator_and_oracle():
    with open(os.path.join(GOLD, "geotext_synth.json")) as f:
        rec = json.load(f)
    import hashlib

    def sha(a):
        return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()

    H = synthetic_graph(rec["n"], rec["edges"])
    assert H.nnz == rec["nnz"]
    assert sha(H.indptr.astype(np.int32)) == rec["sha256_indptr"]
    assert sha(H.indices.astype(np.int32)) == rec["sha256_indices"]
    assert sha(H.data.astype(np.float32)) == rec["sha256_data"]
    Z = dense(rec["n"], rec["K"])
    assert sha(Z) == rec["sha256_Z"]
    Y = O.spmm_f32(H, Z)
    assert sha(Y) == rec["sha256_Y_scipy_f32"]
    assert np.array_equal(Y[rec["sample_rows"]], np.array(rec["Y_sample"], dtype=np.float32))


def test_scatter_add_and_adam():
    out = np.zeros((4, 3), np.float32)
    src = np.arange(15, dtype=np.float32).reshape(5, 3)
    idx = np.array([1, 3, 1, 1, 0])
    ref = np.zeros((4, 3), np.float32)
    np.add.at(ref, idx, src)
    assert np.array_equal(O.scatter_add_f32(out, idx, src), ref)
    st = {}
    p = {"w": np.ones(3)}
    new = O.adam_step(p, {"w": np.array([1.0, -1.0, 0.0])}, st)
    assert np.allclose(new["w"], [1 - 4e-3, 1 + 4e-3, 1.0])


def test_glorot_uniform_is_lasagne_draw_order():
    """layers._glorot_uniform restates lasagne.init.GlorotUniform().sample((n1, n2)):
    uniform(-sqrt(3)*std, sqrt(3)*std) with std = sqrt(2/(n1+n2)) from numpy's global
    stream, floatX'd; two consecutive layers draw W1 then W2 (mlpconv.py:205-217)."""
    from graphconvgeo_amd.layers import _glorot_uniform
    np.random.seed(77)
    W1 = _glorot_uniform(50, 8)
    W2 = _glorot_uniform(8, 3)
    rs = np.random.RandomState(77)
    e1 = rs.uniform(-np.sqrt(3) * np.sqrt(2 / 58), np.sqrt(3) * np.sqrt(2 / 58), (50, 8))
    e2 = rs.uniform(-np.sqrt(3) * np.sqrt(2 / 11), np.sqrt(3) * np.sqrt(2 / 11), (8, 3))
    assert W1.dtype == np.float32 and np.array_equal(W1, e1.astype(np.float32))
    assert np.array_equal(W2, e2.astype(np.float32))
    assert np.array_equal(_glorot_uniform(50, 8, 5), _glorot_uniform(50, 8, np.random.RandomState(5)))
