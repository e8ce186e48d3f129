"""The hot path as registered torch operators (`torch.ops.gcg.*`), with fake kernels.

The reference's `S.dot` is a Theano Op inside a compiled function graph (mlpconv.py:71-73,
90; the graph is compiled by theano.function at mlpconv.py:265-268). The analogue here: every
product of the GCN layers is a `torch.library` custom op whose real kernel is the HIP launch
in libgcg_spmm.so and whose fake kernel states the output's shape, dtype and row stride, so
`torch.compile` / FakeTensor tracing sees through a whole layer stack without graph breaks:

  gcg::spmm_csr(Z, bias?, csr, rows, act, mode, want_gate) -> (Y, gate)
        Y = act(A . Z + bias)[rows] (sparse.spmm); gate = the rectify gate bytes (or empty)
  gcg::spmm_csr_backward(gY, gate, csr, rows, mode, has_gate, want_z, want_bias) -> (gZ, gb)
        Theano's gradient of the above: rectify gate rule, A^T . g / (A[rows])^T . g, colsum
  gcg::gemm_nt(A, Bt, bias?, act) -> C           C = act(A . Bt^T + bias)   (MFMA, LDS-DMA)
  gcg::gemm_tn(A, B, scale?) -> C                C = scale . A^T . B        (split-K MFMA)
  gcg::column_sum(X) -> x                        X.sum(0), deterministic (bias gradients)
  gcg::dense_matmul(A, W, b?) -> C               T.dot(h, W) (+ b), mlpconv.py:88
  gcg::project_softmax_xent(P, W, b?, labels, denom, row_weight?, want_grad) -> (loss, acc, G)
        the fused output layer: softmax(P . W + b) -> mean CE, accuracy, dlogits (mlpconv.py:88-95)

spmm_csr, dense_matmul and project_softmax_xent carry their autograd formulas
(`register_autograd`), whose backward passes are themselves built from these ops. Sparse
operators and row lists are not tensors: a DeviceCSR / RowSelection gets an integer id when it
is created (`sparse._register_object`), and the ops take that id.

The eager training path keeps its autograd.Functions (layers._CSRMatMul, dense._MatMul; same
kernels, plus side-stream weight gradients); `layers.csr_matmul`, `dense.matmul` and
`dense.project_softmax_xent` route through these ops whenever torch.compile is tracing.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
from torch import Tensor

from . import sparse as gs

LIB = "gcg"
_ACTS = ("none", "relu")


def _n_out(csr: int, rows: int) -> int:
    A = gs.registered(csr)
    return A.n_rows if rows < 0 else gs.registered(rows).n


def _dense_like(n: int, k: int, device) -> Tensor:
    """An empty tensor with empty_dense's layout (row stride sparse.row_stride(k))."""
    ld = gs.row_stride(k) if k > 0 else 0
    if ld == k:
        return torch.empty((n, k), dtype=torch.float32, device=device)
    return torch.empty_strided((n, k), (ld, 1), dtype=torch.float32, device=device)


def _gate_like(n: int, k: int, device) -> Tensor:
    ld = (k + 3) // 4 * 4
    if ld == k:
        return torch.empty((n, k), dtype=torch.uint8, device=device)
    return torch.empty_strided((n, k), (ld, 1), dtype=torch.uint8, device=device)


def _rows_arg(rows: int):
    return None if rows < 0 else gs.registered(rows)


# -- gcg::spmm_csr -------------------------------------------------------------------------------
@torch.library.custom_op(f"{LIB}::spmm_csr", mutates_args=())
def spmm_csr_op(Z: Tensor, bias: Optional[Tensor], csr: int, rows: int, act: str, mode: str,
                want_gate: bool) -> Tuple[Tensor, Tensor]:
    A = gs.registered(csr)
    sel = _rows_arg(rows)
    n_out = A.n_rows if sel is None else sel.n
    gate = gs.empty_gate(n_out, Z.shape[1], Z.device) if want_gate else \
        torch.empty(0, dtype=torch.uint8, device=Z.device)
    Y = gs.spmm(A, Z, bias=bias, act=None if act == "none" else act, rows=sel, mode=mode,
                gate=gate if want_gate else None)
    return Y, gate


@spmm_csr_op.register_fake
def _(Z, bias, csr, rows, act, mode, want_gate):
    n_out, K = _n_out(csr, rows), Z.shape[1]
    gate = _gate_like(n_out, K, Z.device) if want_gate else Z.new_empty(0, dtype=torch.uint8)
    return _dense_like(n_out, K, Z.device), gate


@torch.library.custom_op(f"{LIB}::spmm_csr_backward", mutates_args=())
def spmm_csr_backward_op(gY: Tensor, gate: Tensor, csr: int, rows: int, mode: str,
                         has_gate: bool, want_z: bool, want_bias: bool) -> Tuple[Tensor, Tensor]:
    A = gs.registered(csr)
    sel = _rows_arg(rows)
    if gY.stride(-1) != 1:
        gY = gY.contiguous()
    K = gY.shape[1]
    if has_gate and K <= 1024:
        g, g_bias = gs.relu_backward(gY, gate=gate, bias_grad=want_bias)
    elif not has_gate:
        g = gY
        g_bias = (gs.column_sum(gY) if K <= 1024 else gY.sum(dim=0)) if want_bias else None
    else:
        g = gY * (gate.to(gY.dtype) * 0.5)
        g_bias = g.sum(dim=0) if want_bias else None
    g_Z = None
    if want_z:
        g_Z = gs.spmm(A.rows_transpose(sel), g, mode=mode) if sel is not None else \
            A.tmatmul(g, mode=mode)
    empty = gY.new_empty(0)
    return (g_Z if g_Z is not None else empty), (g_bias if g_bias is not None else empty)


@spmm_csr_backward_op.register_fake
def _(gY, gate, csr, rows, mode, has_gate, want_z, want_bias):
    A = gs.registered(csr)
    K = gY.shape[1]
    gZ = _dense_like(A.n_cols, K, gY.device) if want_z else gY.new_empty(0)
    gb = gY.new_empty(K) if want_bias else gY.new_empty(0)
    return gZ, gb


def _spmm_setup(ctx, inputs, output):
    Z, bias, csr, rows, act, mode, want_gate = inputs
    ctx.csr, ctx.rows, ctx.mode = csr, rows, mode
    ctx.has_gate = bool(want_gate)
    ctx.has_bias = bias is not None
    ctx.save_for_backward(output[1])


def _spmm_backward(ctx, gY, _g_gate):
    (gate,) = ctx.saved_tensors
    want_z = ctx.needs_input_grad[0]
    want_b = ctx.has_bias and ctx.needs_input_grad[1]
    gZ, gb = torch.ops.gcg.spmm_csr_backward(gY, gate, ctx.csr, ctx.rows, ctx.mode, ctx.has_gate,
                                             want_z, want_b)
    return (gZ if want_z else None), (gb if want_b else None), None, None, None, None, None


spmm_csr_op.register_autograd(_spmm_backward, setup_context=_spmm_setup)


def spmm_csr(A, Z: Tensor, bias: Optional[Tensor] = None, act: Optional[str] = None,
             rows=None, mode: str = "auto") -> Tensor:
    """Differentiable act(A . Z + bias)[rows] through gcg::spmm_csr (S.dot + epilogue)."""
    act = "none" if act in (None, "none", "linear") else "relu"
    want_gate = act == "relu" and torch.is_grad_enabled() and (
        Z.requires_grad or (bias is not None and bias.requires_grad))
    Y, _gate = torch.ops.gcg.spmm_csr(Z, bias, A.op_id, -1 if rows is None else rows.op_id, act,
                                      mode, want_gate)
    return Y


# -- dense products ------------------------------------------------------------------------------
@torch.library.custom_op(f"{LIB}::gemm_nt", mutates_args=())
def gemm_nt_op(A: Tensor, Bt: Tensor, bias: Optional[Tensor], act: str) -> Tensor:
    from . import dense
    return dense.gemm_nt(A, Bt, bias=bias, act=None if act == "none" else act)


@gemm_nt_op.register_fake
def _(A, Bt, bias, act):
    return _dense_like(A.shape[0], Bt.shape[0], A.device)


@torch.library.custom_op(f"{LIB}::gemm_tn", mutates_args=())
def gemm_tn_op(A: Tensor, B: Tensor, scale: Optional[Tensor]) -> Tensor:
    from . import dense
    return dense.gemm_tn(A, B, scale=scale)


@gemm_tn_op.register_fake
def _(A, B, scale):
    return A.new_empty((A.shape[1], B.shape[1]))


@torch.library.custom_op(f"{LIB}::column_sum", mutates_args=())
def column_sum_op(X: Tensor) -> Tensor:
    """X.sum(0), deterministic (gcg_column_sum_f32, K <= 1024): the bias gradients."""
    return gs.column_sum(X) if X.shape[1] <= 1024 else X.sum(dim=0)


@column_sum_op.register_fake
def _(X):
    return X.new_empty(X.shape[1])


def _padded(W: Tensor, transpose: bool) -> Tensor:
    """[rows, cols] view of a zero-padded [rows, round4(cols)] copy of W (or W^T): the weight
    operand layout of the MFMA kernels, built with traceable torch ops."""
    src = W.t() if transpose else W
    cols = src.shape[1]
    pad = (cols + 3) // 4 * 4 - cols
    return torch.nn.functional.pad(src, (0, pad))[:, :cols] if pad else src.contiguous()


@torch.library.custom_op(f"{LIB}::dense_matmul", mutates_args=())
def dense_matmul_op(A: Tensor, W: Tensor, b: Optional[Tensor]) -> Tensor:
    from . import dense
    return dense.gemm_nt(A, _padded(W, True), bias=b)


@dense_matmul_op.register_fake
def _(A, W, b):
    return _dense_like(A.shape[0], W.shape[1], A.device)


def _mm_setup(ctx, inputs, output):
    A, W, b = inputs
    ctx.has_b = b is not None
    ctx.save_for_backward(A, W)


def _mm_backward(ctx, g):
    A, W = ctx.saved_tensors
    gA = gW = gb = None
    if ctx.needs_input_grad[0]:
        gA = torch.ops.gcg.gemm_nt(g, _padded(W, False), None, "none")  # g . W^T
    if ctx.needs_input_grad[1]:
        gW = torch.ops.gcg.gemm_tn(A, g, None)  # A^T . g
    if ctx.has_b and ctx.needs_input_grad[2]:
        gb = torch.ops.gcg.column_sum(g)
    return gA, gW, gb


dense_matmul_op.register_autograd(_mm_backward, setup_context=_mm_setup)


@torch.library.custom_op(f"{LIB}::project_softmax_xent", mutates_args=())
def project_softmax_xent_op(P: Tensor, W: Tensor, b: Optional[Tensor], labels: Tensor,
                            denom: int, row_weight: Optional[Tensor],
                            want_grad: bool) -> Tuple[Tensor, Tensor, Tensor]:
    from . import dense
    P = dense._aligned_operand(P, "P")
    M, N = P.shape[0], W.shape[1]
    D = float(max(denom, 1))
    y = dense._labels_i32(labels, M, N)
    G = gs.empty_dense(M, N, P.device) if want_grad else P.new_empty(0)
    loss_rows = torch.empty(M, dtype=torch.float32, device=P.device)
    correct = torch.empty(M, dtype=torch.float32, device=P.device)
    dense._fused(P, _padded(W, False), b, y, 1.0 / D, None, G if want_grad else None, loss_rows,
                 correct, None if row_weight is None else row_weight.contiguous())
    return loss_rows.sum() / D, correct.sum() / D, G


@project_softmax_xent_op.register_fake
def _(P, W, b, labels, denom, row_weight, want_grad):
    G = _dense_like(P.shape[0], W.shape[1], P.device) if want_grad else P.new_empty(0)
    return P.new_empty(()), P.new_empty(()), G


def _px_setup(ctx, inputs, output):
    P, W, b, labels, denom, row_weight, want_grad = inputs
    ctx.has_b = b is not None
    ctx.save_for_backward(P, W, output[2])


def _px_backward(ctx, g_loss, _g_acc, _g_G):
    P, W, G = ctx.saved_tensors
    gP = gW = gb = None
    if ctx.needs_input_grad[0]:
        gP = torch.ops.gcg.gemm_nt(G, _padded(W, False) * g_loss, None, "none")  # G . (g W)^T
    if ctx.needs_input_grad[1]:
        gW = torch.ops.gcg.gemm_tn(P, G, g_loss.reshape(1))  # g P^T . G
    if ctx.has_b and ctx.needs_input_grad[2]:
        gb = torch.ops.gcg.column_sum(G) * g_loss
    return gP, gW, gb, None, None, None, None


project_softmax_xent_op.register_autograd(_px_backward, setup_context=_px_setup)


# -- gcg::transform_propagate (the reference order's output layer, re-associated backward) ------
@torch.library.custom_op(f"{LIB}::transform_propagate", mutates_args=())
def transform_propagate_op(h: Tensor, W: Tensor, b: Optional[Tensor], csr: int, rows: int,
                           mode: str) -> Tensor:
    """(S.dot(H, T.dot(h, W)) + b)[rows] (mlpconv.py:88-94) as the reference associates it:
    the NT GEMM, then the C-wide SpMM. The compiled twin of layers._TransformPropagate."""
    from . import dense
    Z = dense.gemm_nt(h, _padded(W, True))
    return gs.spmm(gs.registered(csr), Z, bias=b, rows=_rows_arg(rows), mode=mode)


@transform_propagate_op.register_fake
def _(h, W, b, csr, rows, mode):
    return _dense_like(_n_out(csr, rows), W.shape[1], h.device)


def _tp_setup(ctx, inputs, output):
    h, W, b, csr, rows, mode = inputs
    ctx.csr, ctx.rows, ctx.mode = csr, rows, mode
    ctx.has_b = b is not None
    ctx.save_for_backward(h, W)


def _tp_backward(ctx, g):
    """dh = H[rows]^T . (g . W^T), dW = (H[rows] . h)^T . g, db = colsum(g): the re-associated
    backward of layers._TransformPropagate, from the other ops (the same kernels, bitwise)."""
    h, W = ctx.saved_tensors
    gh = gW = gb = None
    if ctx.has_b and ctx.needs_input_grad[2]:
        gb = torch.ops.gcg.column_sum(g)
    if ctx.needs_input_grad[1]:
        P, _ = torch.ops.gcg.spmm_csr(h, None, ctx.csr, ctx.rows, "none", ctx.mode, False)
        gW = torch.ops.gcg.gemm_tn(P, g, None)
    if ctx.needs_input_grad[0]:
        GW = torch.ops.gcg.gemm_nt(g, _padded(W, False), None, "none")
        gh, _ = torch.ops.gcg.spmm_csr_backward(GW, g.new_empty(0, dtype=torch.uint8), ctx.csr,
                                                ctx.rows, ctx.mode, False, True, False)
    return gh, gW, gb, None, None, None


transform_propagate_op.register_autograd(_tp_backward, setup_context=_tp_setup)


def transform_propagate(h: Tensor, W: Tensor, b: Optional[Tensor], A, rows=None,
                        mode: str = "auto") -> Tensor:
    return torch.ops.gcg.transform_propagate(h, W, b, A.op_id,
                                             -1 if rows is None else rows.op_id, mode)


def dense_matmul(A: Tensor, W: Tensor, b: Optional[Tensor] = None) -> Tensor:
    return torch.ops.gcg.dense_matmul(A, W, b)


def project_softmax_xent(P: Tensor, W: Tensor, b: Optional[Tensor], labels: Tensor,
                         denom: Optional[int] = None, row_weight: Optional[Tensor] = None):
    want = torch.is_grad_enabled() and any(
        t is not None and t.requires_grad for t in (P, W, b))
    loss, acc, _G = torch.ops.gcg.project_softmax_xent(
        P, W, b, labels, int(P.shape[0] if denom is None else denom), row_weight, want)
    return loss, acc
