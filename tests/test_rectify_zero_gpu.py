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


def _gate_of(pre: np.ndarray) -> np.ndarray:
    return (2 * (pre > 0) + (pre == 0)).astype(np.uint8)


def test_gate_bytes_split_rows_fast(cuda):
    """mode='fast' with a small task size: the hub rows are split into segments and the
    spmm_fixup_kernel writes their output and gate bytes. The gate must be the sign of the
    kernel's own pre-activation (same plan, no activation), with exact zeros in the split rows."""
    n, k = 5000, 40
    u, v = uniform_edges(n, 30000, seed=5)
    hubs = np.array([0, 17, 4999])
    hu = np.repeat(hubs, 1500)
    hv = np.concatenate([np.random.default_rng(h).choice(np.arange(n), 1500, replace=False)
                         for h in hubs])
    keep = hu != hv
    H = csr_from_edges(n, np.concatenate([u, hu[keep]]), np.concatenate([v, hv[keep]]))
    A = gs.DeviceCSR.from_scipy(H, cuda, symmetric=True)
    g = torch.Generator(device=cuda).manual_seed(3)
    Z = torch.randn((n, k), device=cuda, generator=g)
    Z[:, :4] = 0.0  # exact-zero pre-activations in every row, the split hub rows included
    b = torch.zeros(k, device=cuda)
    b[4:7] = torch.tensor([1.0, -1.0, 0.0])
    task = 256
    plan = A.plan(None, ordered=False, task_nnz=task)
    assert plan.info()["n_long_rows"] >= len(hubs)  # the fixup path really runs
    pre = gs.spmm(A, Z, bias=b, mode="fast", task_nnz=task).cpu().numpy()
    gate = gs.empty_gate(n, k, cuda)
    Y = gs.spmm(A, Z, bias=b, act="relu", mode="fast", task_nnz=task, gate=gate)
    assert np.array_equal(gate.cpu().numpy(), _gate_of(pre))
    assert np.array_equal(Y.cpu().numpy(), O.relu(pre))
    assert (gate.cpu().numpy()[hubs, :4] == 1).all()
    # and the split rows stay within the 1e-5 bar of the float64 product
    ref = H.astype(np.float64) @ Z.cpu().numpy().astype(np.float64) + b.cpu().numpy()
    assert np.abs(pre - ref).max() < 1e-5


def test_gate_bytes_rowwise_large_row_subset(cuda):
    """The plan-less rowwise launch on >= 65536 output rows (U = 16 per wave there) with a row
    subset: gate bytes and outputs bitwise the oracle's, exact zeros included."""
    n, k = 70000, 24
    u, v = uniform_edges(n, 200000, seed=9)
    H = csr_from_edges(n, u, v)
    A = gs.DeviceCSR.from_scipy(H, cuda, symmetric=True)
    rows = np.random.default_rng(4).choice(n, 66000, replace=True).astype(np.int32)
    g = torch.Generator(device=cuda).manual_seed(5)
    Z = torch.randn((n, k), device=cuda, generator=g)
    Z[:, :3] = 0.0
    b = torch.zeros(k, device=cuda)
    b[3:6] = torch.tensor([0.5, -0.5, 0.0])
    gate = gs.empty_gate(rows.size, k, cuda)
    sel = gs.RowSelection(rows, cuda)
    Y = gs.spmm(A, Z, bias=b, act="relu", rows=sel, mode="rowwise", gate=gate)
    pre = O.spmm_f32(H, Z.cpu().numpy(), bias=b.cpu().numpy())[rows]
    assert np.array_equal(gate.cpu().numpy(), _gate_of(pre))
    assert np.array_equal(Y.cpu().numpy(), O.relu(pre))
    assert (gate.cpu().numpy()[:, :3] == 1).all()
