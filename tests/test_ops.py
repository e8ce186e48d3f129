"""The registered operators (graphconvgeo_amd.ops, torch.ops.gcg.*) on the CPU: schemas and
fake kernels (shape, dtype, row stride) under FakeTensorMode -- no GPU, no kernel launch."""
import pytest
import torch
from torch._subclasses.fake_tensor import FakeTensorMode

from graphconvgeo_amd import ops  # noqa: F401  (registers torch.ops.gcg.*)
from graphconvgeo_amd import sparse as gs


class _Operator:  # stand-in for a DeviceCSR: the fake kernels read only its shape
    def __init__(self, n_rows, n_cols):
        self.n_rows, self.n_cols = n_rows, n_cols
        self.op_id = gs._register_object(self)


class _Rows:  # stand-in for a RowSelection
    def __init__(self, n):
        self.n = n
        self.op_id = gs._register_object(self)


def test_every_op_is_registered():
    for name in ("spmm_csr", "spmm_csr_backward", "gemm_nt", "gemm_tn", "column_sum",
                 "dense_matmul", "project_softmax_xent", "transform_propagate"):
        assert hasattr(torch.ops.gcg, name), name


@pytest.mark.parametrize("K", [1, 3, 64, 300, 930])
def test_spmm_fake_layout_matches_empty_dense(K):
    A, R = _Operator(1000, 800), _Rows(37)
    with FakeTensorMode():
        Z = torch.empty((800, K), device="cuda")
        b = torch.empty(K, device="cuda")
        Y, gate = torch.ops.gcg.spmm_csr(Z, b, A.op_id, -1, "relu", "ordered", True)
        assert Y.shape == (1000, K) and Y.dtype == torch.float32
        assert Y.stride() == ((gs.row_stride(K), 1) if gs.row_stride(K) != K else (K, 1))
        assert gate.dtype == torch.uint8 and gate.shape == (1000, K)
        assert gate.stride(0) == (K + 3) // 4 * 4 or gate.stride(0) == K
        Y2, g2 = torch.ops.gcg.spmm_csr(Z, None, A.op_id, R.op_id, "none", "ordered", False)
        assert Y2.shape == (37, K) and g2.numel() == 0
        gZ, gb = torch.ops.gcg.spmm_csr_backward(Y2, g2, A.op_id, R.op_id, "ordered", False, True,
                                                 True)
        assert gZ.shape == (800, K) and gb.shape == (K,)


def test_dense_fakes():
    with FakeTensorMode():
        P = torch.empty((37, 300), device="cuda")
        W = torch.empty((300, 930), device="cuda")
        C = torch.ops.gcg.dense_matmul(P, W, None)
        assert C.shape == (37, 930) and C.stride() == (gs.row_stride(930), 1)
        y = torch.empty(37, dtype=torch.int32, device="cuda")
        loss, acc, G = torch.ops.gcg.project_softmax_xent(P, W, None, y, 37, None, True)
        assert loss.shape == () and acc.shape == () and G.shape == (37, 930)
        assert torch.ops.gcg.gemm_tn(P, C, None).shape == (300, 930)
        assert torch.ops.gcg.column_sum(C).shape == (930,)


def test_transform_propagate_fake():
    """gcg::transform_propagate, the reference order's output layer: [rows of H] x C."""
    A, R = _Operator(1000, 1000), _Rows(37)
    with FakeTensorMode():
        h = torch.empty((1000, 32), device="cuda")
        W = torch.empty((32, 930), device="cuda")
        b = torch.empty(930, device="cuda")
        Y = torch.ops.gcg.transform_propagate(h, W, b, A.op_id, R.op_id, "ordered")
        assert Y.shape == (37, 930) and Y.stride() == (gs.row_stride(930), 1)
        Y = torch.ops.gcg.transform_propagate(h, W, None, A.op_id, -1, "ordered")
        assert Y.shape == (1000, 930)


def test_unknown_operator_id_raises():
    with pytest.raises(KeyError):
        gs.registered(10**9)
