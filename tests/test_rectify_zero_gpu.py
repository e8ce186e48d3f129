"""Theano's rectify gradient at an exactly-zero pre-activation (mlpconv.py:75-77).

lasagne.nonlinearities.rectify is theano.tensor.nnet.relu = 0.5*(x + |x|); its gradient is
0.5*g*(1 + sgn(x)), so g/2 where the pre-activation is exactly 0. That happens for an isolated
user (H row = its self loop only, tensormain.py:170-180) with an empty bag-of-words row and
b1 = 0 (Lasagne's Constant(0.) default): its whole pre-activation row is 0. The oracle's
float64 backward (gcn_oracle.gcn_backward) encodes the rule; the HIP path carries it in the
gate bytes of the SpMM epilogue (sparse.spmm(gate=...), gcg_relu_backward_gate_f32)."""
import numpy as np
import pytest
import scipy.sparse as sps
import torch

from graphconvgeo_amd import sparse as gs
from graphconvgeo_amd.graph import csr_from_edges
from graphconvgeo_amd.layers import GCN
from graphconvgeo_amd.synth import glorot_uniform, synthetic_features, uniform_edges
from oracle import gcn_oracle as O

pytestmark = pytest.mark.gpu


def isolated_problem(n=3000, n_iso=150, e=20000, f=400, k=32, c=7):
    u, v = uniform_edges(n - n_iso, e)
    H = csr_from_edges(n, u, v)  # nodes [n - n_iso, n) have only their self loop
    iso = np.arange(n - n_iso, n)
    X = synthetic_features(n, f, nnz_per_row=16)
    keep = np.ones(n, np.float32)
    keep[iso] = 0.0
    X = sps.csr_matrix(sps.diags(keep) @ X, dtype=np.float32)
    X.eliminate_zeros()
    X.sort_indices()
    idx = np.concatenate([np.random.default_rng(1).choice(n - n_iso, 1200), iso]).astype(np.int32)
    y = np.random.default_rng(2).integers(0, c, size=idx.size)
    return H, X, iso, idx, y, glorot_uniform(f, k), glorot_uniform(k, c, seed=4)


def test_gate_bytes(cuda):
    H, X, iso, idx, y, W1, W2 = isolated_problem()
    A = gs.DeviceCSR.from_scipy(H, cuda, symmetric=True)
    Z = torch.randn((H.shape[0], 32), device=cuda)
    Z[torch.as_tensor(iso, device=cuda)] = 0.0
    b = torch.zeros(32, device=cuda)
    b[:3] = torch.tensor([1.0, -1.0, 0.0])
    gate = gs.empty_gate(H.shape[0], 32, cuda)
    Y = gs.spmm(A, Z, bias=b, act="relu", mode="ordered", gate=gate)
    pre = O.spmm_f32(H, Z.cpu().numpy(), bias=b.cpu().numpy())
    want = (2 * (pre > 0) + (pre == 0)).astype(np.uint8)
    assert np.array_equal(gate.cpu().numpy(), want)
    assert np.array_equal(Y.cpu().numpy(), O.relu(pre))
    assert (want[iso] == 1).sum() > 0  # the isolated rows really are exact zeros


@pytest.mark.parametrize("mode", ["ordered", "fast"])
def test_isolated_nodes_bias_gradient(cuda, mode):
    H, X, iso, idx, y, W1, W2 = isolated_problem()
    n, f = X.shape
    k, c = W2.shape
    b1, b2 = np.zeros(k, np.float32), np.zeros(c, np.float32)
    model = GCN(H, X, f, k, c, device=cuda, W1=W1, W2=W2, mode=mode)
    P = model(idx)
    loss = torch.nn.functional.nll_loss(torch.log(P), torch.from_numpy(y).to(cuda))
    loss.backward()
    fwd = O.gcn_forward(X, H, W1, b1, W2, b2, idx)
    assert np.all(fwd["pre1"][iso] == 0.0)
    gr = O.gcn_backward(X, H, W1, W2, fwd, idx, y, regul_coefs=(0.0, 0.0))
    got_b1 = model.l_hid1.b.grad.cpu().numpy()
    tol = 1e-5 * max(1.0, np.abs(gr["b1"]).max())
    assert np.abs(got_b1 - gr["b1"]).max() < tol
    # the isolated rows' half-gradients (gr["pre1"] holds g/2 there) are what the rule
    # changes: a mask on output > 0 would drop this whole contribution to db1
    contrib = gr["pre1"][iso].sum(axis=0)
    assert np.abs(contrib).max() > 100 * tol
    got_W1 = model.l_hid1.W.grad.cpu().numpy()
    assert np.abs(got_W1 - gr["W1"]).max() < 1e-5 * max(1.0, np.abs(gr["W1"]).max())
