"""Mention-graph construction vs the reference's own get_graph output (golden fixture).

CPU: the host parser (graphconvgeo_amd.mentions) + the oracle projection reproduce the
reference's projected edges. GPU: gcg_project_mention_graph and the full chain to H."""
import importlib.util
import os

import numpy as np
import pytest

from graphconvgeo_amd.mentions import mention_incidences
from oracle import gcn_oracle as O

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _tables():
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(GOLD, "make_golden.py"))
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)  # module import does not touch /root/reference
    return mg.mention_tables()


@pytest.fixture(scope="module")
def gold():
    return dict(np.load(os.path.join(GOLD, "mention_graph.npz")))


def test_host_parser_and_oracle_projection_match_reference(gold):
    n_users, n_nodes, a, b = mention_incidences(*_tables())
    assert n_users == int(gold["n"])
    assert n_nodes > n_users  # external mention names got their own ids
    edges = O.project_mentions(n_users, n_nodes, a, b, celebrity_threshold=10)
    assert np.array_equal(edges, gold["edges"].astype(np.int64))


def test_oracle_projection_properties():
    # users 0..3; mention node 4 shared by 0,1,2 (clique); node 5 seen once (dropped);
    # node 6 mentioned by 4 users > threshold 3 (celebrity, dropped); 3 mentions 2 directly.
    a = [4, 4, 4, 5, 6, 6, 6, 6, 2]
    b = [0, 1, 2, 3, 0, 1, 2, 3, 3]
    e = O.project_mentions(4, 7, a, b, celebrity_threshold=3)
    assert e.tolist() == [[0, 1], [0, 2], [1, 2], [2, 3]]


@pytest.mark.gpu
def test_device_projection_matches_reference(cuda, gold):
    from graphconvgeo_amd.mentions import mention_graph_operator, project_mentions
    tables = _tables()
    n_users, n_nodes, a, b = mention_incidences(*tables)
    u, v = project_mentions(n_users, n_nodes, a, b, 10, cuda)
    got = np.stack([u.cpu().numpy(), v.cpu().numpy()], axis=1)
    assert np.array_equal(got, gold["edges"])
    H = mention_graph_operator(*tables, celebrity_threshold=10, device=cuda).to_scipy()
    assert np.array_equal(H.indptr, gold["H_indptr"]) and np.array_equal(H.indices, gold["H_indices"])
    assert np.array_equal(H.data, gold["H32_data"])  # bitwise the reference's float32 H


@pytest.mark.gpu
@pytest.mark.parametrize("thr", [1, 2, 5, 30])
def test_device_projection_random(cuda, thr):
    from graphconvgeo_amd.mentions import project_mentions
    rng = np.random.default_rng(thr)
    n_users, n_ment = 3000, 1500
    n_inc = 12000
    a = rng.integers(0, n_users + n_ment, n_inc).astype(np.int32)
    # a few hub users / mentions with many incidences
    a[:300] = 7
    a[300:360] = n_users + 3
    b = rng.integers(0, n_users, n_inc).astype(np.int32)
    u, v = project_mentions(n_users, n_users + n_ment, a, b, thr, cuda)
    got = np.stack([u.cpu().numpy(), v.cpu().numpy()], axis=1).astype(np.int64)
    ref = O.project_mentions(n_users, n_users + n_ment, a, b, thr)
    assert np.array_equal(got, ref)
