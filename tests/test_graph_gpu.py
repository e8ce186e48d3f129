"""GPU graph-operator construction (tensormain.py:170-180) vs the oracle and the fixtures."""
import os

import numpy as np
import pytest
import scipy.sparse as sps

from graphconvgeo_amd.graph import csr_from_edges, normalize_edges_device
from graphconvgeo_amd.synth import powerlaw_edges, uniform_edges
from oracle import gcn_oracle as O

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_device_normalization_matches_reference_fixture(cuda):
    g = dict(np.load(os.path.join(GOLD, "mention_graph.npz")))
    n = int(g["n"])
    edges = g["edges"]
    H = normalize_edges_device(n, edges[:, 0], edges[:, 1], cuda).to_scipy()
    assert np.array_equal(H.indptr, g["H_indptr"])
    assert np.array_equal(H.indices, g["H_indices"])
    assert np.array_equal(H.data, g["H32_data"])  # bitwise: reference H.astype(float32)


@pytest.mark.parametrize("kind", ["powerlaw", "uniform"])
def test_device_normalization_large(cuda, kind):
    n, e = 200_000, 1_500_000
    u, v = (powerlaw_edges if kind == "powerlaw" else uniform_edges)(n, e)
    # shuffle + flip some edges and add duplicates: the device path must canonicalize
    rng = np.random.default_rng(1)
    p = rng.permutation(e)
    u, v = u[p], v[p]
    flip = rng.random(e) < 0.5
    u2, v2 = np.where(flip, v, u), np.where(flip, u, v)
    dup = rng.choice(e, size=1000)
    u2 = np.concatenate([u2, v2[dup]])
    v2 = np.concatenate([v2, u2[dup]])
    H = normalize_edges_device(n, u2, v2, cuda).to_scipy()
    ref = csr_from_edges(n, u, v)
    assert H.nnz == 2 * e + n
    assert np.array_equal(H.indptr, ref.indptr)
    assert np.array_equal(H.indices, ref.indices)
    assert np.array_equal(H.data, ref.data)
    # and the oracle's independent restatement (lil setdiag path)
    adj = sps.csr_matrix((np.ones(e), (u, v)), shape=(n, n))
    Ho = O.normalize_adjacency(adj + adj.T)
    assert np.array_equal(H.data, Ho.data)


def test_device_normalization_errors(cuda):
    with pytest.raises(ValueError, match="out of range"):
        normalize_edges_device(5, [0, 1], [1, 7], cuda)
    H = normalize_edges_device(4, [], [], cuda).to_scipy()  # isolated nodes: identity
    assert np.array_equal(H.toarray(), np.eye(4, dtype=np.float32))
