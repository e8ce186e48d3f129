"""The hot path as registered torch ops on the GPU (graphconvgeo_amd.ops): torch.library.opcheck
of the real kernels against their schemas / fake kernels / autograd registration, and
torch.compile of the GCN forward (+ backward) with no graph break on the gcg ops, bitwise
equal to the eager autograd.Function path in 'ordered' mode -- the analogue of the reference's
Theano-compiled S.dot graph (mlpconv.py:71-73, 265-268). backend='aot_eager': AOTAutograd
traces through the fake kernels and the registered autograd formulas; no generated kernels."""
import numpy as np
import pytest
import torch

from graphconvgeo_amd import ops  # noqa: F401
from graphconvgeo_amd import sparse as gs
from graphconvgeo_amd.layers import GCN
from graphconvgeo_amd.synth import glorot_uniform, synthetic_features, synthetic_graph

pytestmark = pytest.mark.gpu

OPCHECK = ("test_schema", "test_autograd_registration", "test_faketensor",
           "test_aot_dispatch_static")


def _problem(n=3000, e=20000, f=200, k=32, c=40):
    H = synthetic_graph(n, e)
    X = synthetic_features(n, f, nnz_per_row=16)
    idx = np.random.default_rng(5).choice(n, 900).astype(np.int32)  # duplicates included
    return H, X, idx, glorot_uniform(f, k), glorot_uniform(k, c, seed=4)


def test_opcheck_spmm_csr(cuda):
    H, X, idx, W1, W2 = _problem()
    A = gs.DeviceCSR.from_scipy(H, cuda, symmetric=True)
    rows = gs.RowSelection(idx, cuda)
    Z = torch.randn((H.shape[0], 32), device=cuda, requires_grad=True)
    b = torch.randn(32, device=cuda, requires_grad=True)
    torch.library.opcheck(torch.ops.gcg.spmm_csr.default,
                          (Z, b, A.op_id, -1, "relu", "ordered", True), test_utils=OPCHECK)
    torch.library.opcheck(torch.ops.gcg.spmm_csr.default,
                          (Z, None, A.op_id, rows.op_id, "none", "ordered", False),
                          test_utils=OPCHECK)


def test_opcheck_dense(cuda):
    g = torch.Generator(device=cuda).manual_seed(1)
    P = torch.randn((257, 300), device=cuda, generator=g, requires_grad=True)
    W = (torch.rand((300, 130), device=cuda, generator=g) - 0.5).requires_grad_()
    b = torch.randn(130, device=cuda, generator=g, requires_grad=True)
    y = torch.randint(0, 130, (257,), device=cuda, generator=g, dtype=torch.int32)
    torch.library.opcheck(torch.ops.gcg.dense_matmul.default, (P, W, b), test_utils=OPCHECK)
    torch.library.opcheck(torch.ops.gcg.project_softmax_xent.default,
                          (P, W, b, y, 257, None, True), test_utils=OPCHECK)


@pytest.mark.parametrize("operator", ["symmetric", "rownorm"])
@pytest.mark.parametrize("order", ["reference", "propagate_first"])
def test_compiled_gcn_forward_backward_bitwise_eager(cuda, order, operator):
    """Reference order with C > K (here 40 > 32): eager runs layers._TransformPropagate (the
    re-associated backward) and the compiled graph its registered twin gcg::transform_propagate,
    built from the same kernels -- bitwise equal, forward and every gradient. Also on the
    reference's non-symmetric row-normalized operator (main.py:451-456), whose backward runs
    through CSR(H^T) in both forms."""
    import torch._dynamo as dynamo

    H, X, idx, W1, W2 = _problem()
    if operator == "rownorm":
        from oracle import gcn_oracle as O
        A = H.copy()
        A.data[:] = 1.0
        H = O.row_normalize_l1(A)
    model = GCN(H, X, 200, 32, 40, device=cuda, W1=W1, W2=W2, mode="ordered")
    model.l_out.order = order
    rows = gs.RowSelection(idx, cuda)
    eager = model(rows)
    eager.log().sum().backward()
    eager = eager.detach()  # let the eager autograd graph (and its AccumulateGrad nodes) go
    g_eager = [p.grad.clone() for p in model.parameters()]
    model.zero_grad(set_to_none=True)

    dynamo.reset()
    counters = dynamo.utils.counters
    counters.clear()
    compiled = torch.compile(model.forward, backend="aot_eager", fullgraph=True)  # no breaks
    got = compiled(rows)
    assert torch.equal(got, eager)  # ordered mode: every kernel the same, bit for bit
    got.log().sum().backward()
    for p, ge in zip(model.parameters(), g_eager):
        assert torch.equal(p.grad, ge)
    assert sum(counters["graph_break"].values()) == 0
    assert model.l_hid1.H.symmetric is (operator == "symmetric")
    dynamo.reset()
