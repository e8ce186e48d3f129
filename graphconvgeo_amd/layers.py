"""Graph-convolution layers with the reference's Lasagne plugin signatures (mlpconv.py:59-95).

Reference (Lasagne `Layer` subclasses, Theano graph, host CPU):

    SparseConvolutionDenseLayer(incoming, H=None, num_units, W=GlorotUniform(),
                                b=Constant(0.), nonlinearity=rectify)          mlpconv.py:59-77
        get_output_for(X) = nonlinearity(S.dot(H, S.dot(X, W)) + b);  X must be sparse
    ConvolutionDenseLayer(incoming, H=None, num_units, W=GlorotUniform(), b=Constant(0.),
                          nonlinearity=rectify)  (MLPCONV passes softmax)   mlpconv.py:79-95
        get_output_for(h, target_indices=idx) = nonlinearity((S.dot(H, T.dot(h, W)) + b)[idx])

Here: torch modules with the same constructor arguments and `get_output_for` /
`forward(input, target_indices=None)`. The sparse products run in the HIP kernels
(graphconvgeo_amd.sparse.spmm) with bias + rectify + the target-row subset fused in the
epilogue; the dense projection T.dot(h, W) runs on the hand-written f32 MFMA kernels of csrc/dense.hip
(forward and input gradient on the LDS-DMA NT GEMM, the weight gradient on the split-K
kernel; the trainer's output layer is one fused MFMA kernel, graphconvgeo_amd.dense). Backward follows Theano's rules: grad of
S.dot(A, Z) w.r.t. Z is A^T . gz (A^T = H when H is symmetric -- checked once on the device,
DeviceCSR.check_symmetric -- else CSR(H^T); CSR(X^T) built once on the device), grad of Y[idx]
is a deterministic scatter-add (duplicates add, tensormain.py:226).

`GraphConvLayer` is the name BASELINE.json's north_star uses; it is the generic form.
Rectify is Theano's 0.5*(x+|x|) in the forward, and its gradient 0.5*g*(1+sgn(x)) in the
backward -- g/2 at an exactly-zero pre-activation -- from the gate bytes the SpMM epilogue
writes (sparse.spmm(gate=...)).

Weights default to Lasagne's GlorotUniform drawn from numpy's global stream (W1 then W2 in
MLPCONV, as the reference's DenseLayer constructors draw them), so `np.random.seed(77)`
before the model (tensormain.py:227) starts from the reference's weights.
"""
from __future__ import annotations

from typing import Optional, Union

import numpy as np
import scipy.sparse as sps
import torch
import torch.nn as nn

from . import dense
from . import ops as _ops  # registers torch.ops.gcg.* (the compiled path)
from . import sparse as gs

_FUSED_ACTS = {"rectify": "relu", "relu": "relu"}


def _glorot_uniform(fan_in: int, fan_out: int, rng=None) -> np.ndarray:
    """lasagne.init.GlorotUniform(gain=1.0).sample((num_inputs, num_units)), the default W of
    a Lasagne DenseLayer (mlpconv.py:208; ConvolutionDenseLayer's default at mlpconv.py:214):
    std = gain * sqrt(2 / ((n1 + n2) * receptive_field_size)); Uniform(std=std) draws
    uniform(low=0 - sqrt(3)*std, high=0 + sqrt(3)*std, size) from lasagne.random.get_rng(),
    which is numpy's global stream unless set, then floatX (float32). [recalled Lasagne 0.2;
    Lasagne is not importable here, so this draw order is parity-unpinned.]

    rng: None -> numpy's global stream (np.random; main_mlpconv seeds it with
    np.random.seed(77), tensormain.py:227, before MLPCONV draws W1 then W2), an int seed, or a
    numpy RandomState / Generator."""
    if rng is None:
        rng = np.random.mtrand._rand
    elif isinstance(rng, (int, np.integer)):
        rng = np.random.RandomState(int(rng))
    n1, n2 = int(fan_in), int(fan_out)
    receptive_field_size = np.prod(())  # 1.0: DenseLayer weights are 2-D
    std = 1.0 * np.sqrt(2.0 / ((n1 + n2) * receptive_field_size))
    a, b = 0.0 - np.sqrt(3) * std, 0.0 + np.sqrt(3) * std
    return np.asarray(rng.uniform(low=a, high=b, size=(n1, n2)), dtype=np.float32)


def _as_tensor(x, shape, device) -> torch.Tensor:
    t = torch.as_tensor(np.asarray(x, dtype=np.float32) if not isinstance(x, torch.Tensor) else x,
                        dtype=torch.float32)
    if tuple(t.shape) != tuple(shape):
        raise ValueError(f"expected parameter of shape {shape}, got {tuple(t.shape)}")
    return t.to(device).contiguous()


def _num_inputs(incoming) -> int:
    if isinstance(incoming, int):
        return incoming
    if isinstance(incoming, (tuple, list)):
        return int(incoming[-1])
    if hasattr(incoming, "num_units"):
        return int(incoming.num_units)
    raise ValueError("incoming must be an int (num inputs), a shape tuple or a layer")


def _upload_cached(cache: dict, x, device) -> gs.DeviceCSR:
    """Upload a host sparse input once and reuse it while the same object is passed
    (the reference feeds the same X to every epoch, mlpconv.py:294-295). The cache holds
    a weak reference, so a new matrix that reuses a freed object's id() is re-uploaded."""
    if isinstance(x, gs.DeviceCSR):
        return x
    import weakref

    ref = cache.get("ref")
    if ref is not None and ref() is x and cache.get("sig") == (x.shape, x.nnz):
        return cache["dev"]
    dev = gs.DeviceCSR.from_scipy(x, device)
    cache.clear()
    cache.update(ref=weakref.ref(x), sig=(x.shape, x.nnz), dev=dev)
    return dev


def _as_device_csr(m, device) -> gs.DeviceCSR:
    if isinstance(m, gs.DeviceCSR):
        return m
    if sps.issparse(m):
        return gs.DeviceCSR.from_scipy(m, device)
    raise ValueError("Input for this layer must be sparse")


class _CSRMatMul(torch.autograd.Function):
    """Y = act(A . Z + bias)[rows]; differentiable in Z and bias (S.dot + epilogue)."""

    @staticmethod
    def forward(ctx, Z, bias, A: gs.DeviceCSR, act, rows, mode):
        gate = None
        if act == "relu" and any(ctx.needs_input_grad[:2]):
            # rectify gate (2/1/0 for pre-activation > 0, == 0, < 0) written by the SpMM
            # epilogue: Theano's relu gradient is g/2 at an exact-zero pre-activation
            # (e.g. an isolated node with an empty X row and b = 0), which the output
            # alone cannot tell from a negative one
            n_out = A.n_rows if rows is None else len(rows)
            gate = gs.empty_gate(n_out, Z.shape[1], A.device)
        Y = gs.spmm(A, Z, bias=bias, act=act, rows=rows, mode=mode, gate=gate)
        ctx.A, ctx.act, ctx.rows, ctx.mode = A, act, rows, mode
        ctx.has_bias = bias is not None
        ctx.save_for_backward(gate)
        return Y

    @staticmethod
    def backward(ctx, gY):
        A, rows = ctx.A, ctx.rows
        (gate,) = ctx.saved_tensors
        want_bias = ctx.has_bias and ctx.needs_input_grad[1]
        if gate is not None and gY.shape[1] <= 1024:
            # Theano rectify gradient and bias gradient in one pass (gcg_relu_backward_gate_f32)
            g, g_bias = gs.relu_backward(gY.contiguous() if gY.stride(-1) != 1 else gY,
                                         gate=gate, bias_grad=want_bias)
        elif gate is None:
            g = gY
            g_bias = (gs.column_sum(gY) if gY.shape[1] <= 1024 else gY.sum(dim=0)) \
                if want_bias else None
        else:
            g = gY * (gate.to(gY.dtype) * 0.5)
            g_bias = g.sum(dim=0) if want_bias else None
        g_Z = None
        if ctx.needs_input_grad[0]:
            if rows is not None:
                # (A[rows])^T . g: one SpMM over the targets' nonzeros (sparse.rows_transpose),
                # equal to A^T . inc_subtensor(zeros, rows, g) (mlpconv.py:94, Theano's grad)
                # within fp32 rounding
                # (a row-padded g -- C = 930 columns in 960-float rows -- is passed as is:
                # .contiguous() would copy it and lose the padding the 16-B gathers use)
                g_Z = gs.spmm(A.rows_transpose(rows), g if g.stride(-1) == 1 else g.contiguous(),
                              mode=ctx.mode)
            else:
                g_Z = A.tmatmul(g if g.stride(-1) == 1 else g.contiguous(), mode=ctx.mode)
        return g_Z, g_bias, None, None, None, None


def _index_csr_cached(rows: gs.RowSelection, n_rows: int):
    cache = rows.__dict__.setdefault("_index_csr", {})
    if n_rows not in cache:
        cache[n_rows] = gs.index_csr(rows.device_rows, n_rows)
    return cache[n_rows]


def csr_matmul(A: gs.DeviceCSR, Z: torch.Tensor, bias: Optional[torch.Tensor] = None,
               act: Optional[str] = None, rows: Optional[gs.RowSelection] = None,
               mode: str = "auto") -> torch.Tensor:
    """Differentiable S.dot(A, Z) (+ bias, rectify, row subset) through the HIP kernels.
    Under torch.compile the registered op gcg::spmm_csr (graphconvgeo_amd.ops: same kernels,
    a fake kernel for tracing, its autograd formula made of gcg ops) stands in for the
    autograd.Function."""
    if torch.compiler.is_compiling():
        return _ops.spmm_csr(A, Z, bias, act, rows, mode)
    return _CSRMatMul.apply(Z, bias, A, act, rows, mode)


def _resolve_nonlinearity(nl):
    """Returns (fused kernel activation or None, post-op callable or None)."""
    if nl is None or nl in ("linear", "identity"):
        return None, None
    if isinstance(nl, str):
        if nl in _FUSED_ACTS:
            return _FUSED_ACTS[nl], None
        if nl == "softmax":
            return None, lambda x: torch.softmax(x, dim=1)
        if nl == "tanh":
            return None, torch.tanh
        if nl == "sigmoid":
            return None, torch.sigmoid
        raise ValueError(f"unknown nonlinearity {nl!r}")
    if nl is torch.relu or nl is torch.nn.functional.relu:
        return "relu", None
    return None, nl


class GraphConvLayer(nn.Module):
    """nonlinearity((H . (input . W) + b)[target_indices]) -- one graph-convolution layer.

    input: sparse (scipy / DeviceCSR; X . W runs in the HIP SpMM) or dense torch tensor
    (X . W is an fp32 GEMM). H: scipy sparse or DeviceCSR, uploaded once and shared.
    """

    def __init__(self, incoming=None, H=None, num_units: int = None, W=None, b=0.0,
                 nonlinearity="rectify", device: Union[str, torch.device] = "cuda",
                 mode: str = "auto", require_sparse_input: bool = False, rng=None,
                 in_features: Optional[int] = None):
        super().__init__()
        if num_units is None:
            raise ValueError("num_units is required")
        if H is None:
            raise ValueError("H (the normalized adjacency) is required")
        self.device = torch.device(device)
        self.num_inputs = in_features if in_features is not None else _num_inputs(incoming)
        self.num_units = int(num_units)
        # H^T for the backward: H itself when H is symmetric (declared by its builder, or found
        # so by DeviceCSR.check_symmetric at the first backward), else the built transpose
        self.H = _as_device_csr(H, self.device)
        w = _glorot_uniform(self.num_inputs, self.num_units, rng) if W is None else W
        self.W = nn.Parameter(_as_tensor(w, (self.num_inputs, self.num_units), self.device))
        if b is None:
            self.b = None
        else:
            bb = np.full(self.num_units, float(b), np.float32) if np.isscalar(b) else b
            self.b = nn.Parameter(_as_tensor(bb, (self.num_units,), self.device))
        self.fused_act, self.post = _resolve_nonlinearity(nonlinearity)
        self.mode = mode
        self.require_sparse_input = require_sparse_input
        self._sparse_inputs = {}

    def _sparse_input(self, x) -> gs.DeviceCSR:
        return _upload_cached(self._sparse_inputs, x, self.device)

    def forward(self, input, target_indices=None, **kwargs):
        is_sparse = isinstance(input, gs.DeviceCSR) or sps.issparse(input)
        if self.require_sparse_input and not is_sparse:
            raise ValueError("Input for this layer must be sparse")  # mlpconv.py:67-69
        if is_sparse:
            Z = csr_matmul(self._sparse_input(input), self.W, mode=self.mode)  # S.dot(X, W)
        else:
            Z = dense.matmul(input, self.W)  # T.dot(h, W), mlpconv.py:88 (dW: split-K MFMA)
        rows = None
        if target_indices is not None:
            rows = target_indices if isinstance(target_indices, gs.RowSelection) else \
                gs.RowSelection(target_indices, self.device)
        Y = csr_matmul(self.H, Z, self.b, self.fused_act, rows, self.mode)
        return self.post(Y) if self.post is not None else Y

    # Lasagne-style API
    def get_output_for(self, input, **kwargs):
        return self.forward(input, **kwargs)

    def get_params(self):
        return [p for p in (self.W, self.b) if p is not None]


class SparseConvolutionDenseLayer(GraphConvLayer):
    """mlpconv.py:59-77: nonlinearity(S.dot(H, S.dot(X, W)) + b); X must be sparse."""

    def __init__(self, incoming=None, H=None, num_units=None, W=None, b=0.0,
                 nonlinearity="rectify", **kw):
        super().__init__(incoming, H=H, num_units=num_units, W=W, b=b,
                         nonlinearity=nonlinearity, require_sparse_input=True, **kw)


class _TransformPropagate(torch.autograd.Function):
    """Y = (H . (h . W) + b)[rows]: ConvolutionDenseLayer in the reference order (mlpconv.py:
    88-94) with a backward re-associated for the wide output (round 5).

    Forward exactly as the reference associates it: Z = h . W on the NT GEMM (T.dot(h, W)),
    then the C-wide SpMM (S.dot(H, Z) + b)[rows]. Theano's backward goes through the C-wide
    dZ = H[rows]^T . g -- a C-wide transpose SpMM, then dh = dZ . W^T and dW = h^T . dZ over
    every node. The same linear maps, re-associated:
        dh = H[rows]^T . (g . W^T)      the NT GEMM over the target rows only, the SpMM K wide
        dW = (H[rows] . h)^T . g        a K-wide SpMM over the target rows, the split-K
                                        reduction over the target rows only (side stream)
        db = colsum(g)
    Equal in exact arithmetic; in fp32 within the same float64 bars as the reference
    association (tests/test_config3_gpu.py, test_layers_gpu.py). Used when C > K (World: C =
    930, K = 300: two K-wide SpMMs over the targets' nonzeros instead of one C-wide)."""

    @staticmethod
    def forward(ctx, h, W, b, H: gs.DeviceCSR, rows, mode, slot, proj):
        Z = dense.gemm_nt(h, proj.fwd.get(W, True))  # T.dot(h, W), mlpconv.py:88
        Y = gs.spmm(H, Z, bias=None if b is None else b.detach(), rows=rows, mode=mode)
        ctx.save_for_backward(h, W)
        ctx.H, ctx.rows, ctx.mode, ctx.slot, ctx.proj = H, rows, mode, slot, proj
        ctx.has_b = b is not None
        return Y

    @staticmethod
    def backward(ctx, g):
        h, W = ctx.saved_tensors
        H, rows, mode = ctx.H, ctx.rows, ctx.mode
        g = g if g.stride(-1) == 1 else g.contiguous()
        gh = gW = gb = None
        if ctx.has_b and ctx.needs_input_grad[2]:
            gb = dense._colsum(g)
        if ctx.needs_input_grad[1]:
            P = gs.spmm(H, h, rows=rows, mode=mode)  # (H . h)[rows], K wide
            if ctx.slot is not None:  # the split-K reduction on the side stream
                ctx.slot.args = (P, g, None)
                gW = dense._placeholder_grad(W, g)
            else:
                gW = dense.gemm_tn(P, g)
        if ctx.needs_input_grad[0]:
            GW = dense.gemm_nt(g, ctx.proj.bwd.get(W, False))  # g . W^T over the target rows
            T = H.rows_transpose(rows) if rows is not None else None
            gh = gs.spmm(T, GW, mode=mode) if T is not None else H.tmatmul(GW, mode=mode)
        return gh, gW, gb, None, None, None, None, None


# reference order, C > K: the re-associated backward of _TransformPropagate (False: autograd
# through dense.matmul + csr_matmul, Theano's association -- A/B and tests)
REASSOCIATED_BACKWARD = True


class ConvolutionDenseLayer(GraphConvLayer):
    """mlpconv.py:79-95: nonlinearity((S.dot(H, T.dot(h, W)) + b)[target_indices]).

    The default nonlinearity is rectify, Lasagne DenseLayer's default (the class only adds H);
    MLPCONV passes softmax explicitly (mlpconv.py:214-217).

    order: "reference" -- transform then propagate, as mlpconv.py:88-90 (default);
           "propagate_first" -- ((H . h)[target_indices]) . W + b: the SpMM runs at the
           input width K instead of num_units C and only for the target rows, and its
           backward SpMM is K wide too (C = 930 vs K = 300 on Twitter-World). Equal in exact
           arithmetic; in fp32 within the 1e-5 bar, not bitwise to the reference order;
           "auto" -- propagate_first when num_units > num_inputs.
    """

    def __init__(self, incoming=None, H=None, num_units=None, W=None, b=0.0,
                 nonlinearity="rectify", order: str = "reference", **kw):
        super().__init__(incoming, H=H, num_units=num_units, W=W, b=b,
                         nonlinearity=nonlinearity, **kw)
        if order not in ("reference", "propagate_first", "auto"):
            raise ValueError("order must be 'reference', 'propagate_first' or 'auto'")
        if order == "auto":
            order = "propagate_first" if self.num_units > self.num_inputs else "reference"
        self.order = order

    def propagate(self, input, target_indices=None) -> torch.Tensor:
        """(H . h)[target_indices] -- the K-wide SpMM of the propagate-first order."""
        rows = None
        if target_indices is not None:
            rows = target_indices if isinstance(target_indices, gs.RowSelection) else \
                gs.RowSelection(target_indices, self.device)
        return csr_matmul(self.H, input, None, None, rows, self.mode)

    def forward(self, input, target_indices=None, **kwargs):
        sparse_in = isinstance(input, gs.DeviceCSR) or sps.issparse(input)
        if (self.order == "reference" and not sparse_in and REASSOCIATED_BACKWARD
                and self.fused_act is None and self.num_units > self.num_inputs
                and torch.is_grad_enabled()):
            rows = None
            if target_indices is not None:
                rows = target_indices if isinstance(target_indices, gs.RowSelection) else \
                    gs.RowSelection(target_indices, self.device)
            if torch.compiler.is_compiling():  # the registered twin (graphconvgeo_amd.ops)
                Y = _ops.transform_propagate(input, self.W, self.b, self.H, rows, self.mode)
                return self.post(Y) if self.post is not None else Y
            proj = dense.projection_of(self.W)
            Wa, slot = dense._weight_on_side_stream(self.W)
            Y = _TransformPropagate.apply(input, Wa, self.b, self.H, rows, self.mode, slot, proj)
            return self.post(Y) if self.post is not None else Y
        if self.order == "reference" or sparse_in:
            return super().forward(input, target_indices=target_indices, **kwargs)
        P = self.propagate(input, target_indices)  # (H . h)[rows], K wide
        Y = dense.matmul(P, self.W, self.b)
        if self.fused_act == "relu":
            Y = torch.relu(Y)
        return self.post(Y) if self.post is not None else Y


class SparseInputDenseLayer(nn.Module):
    """lasagne_layers.py:20-29 (and mlpconv.py:27-36): nonlinearity(S.dot(X, W) + b), X sparse.

    The input layer of the MDN heads (lang2loc.py:285); the same HIP SpMM (X . W gathers
    rows of W) with bias + rectify fused. Lasagne's DenseLayer default nonlinearity is
    rectify."""

    def __init__(self, incoming=None, num_units: int = None, W=None, b=0.0,
                 nonlinearity="rectify", device: Union[str, torch.device] = "cuda",
                 mode: str = "auto", rng=None, in_features: Optional[int] = None):
        super().__init__()
        if num_units is None:
            raise ValueError("num_units is required")
        self.device = torch.device(device)
        self.num_inputs = in_features if in_features is not None else _num_inputs(incoming)
        self.num_units = int(num_units)
        w = _glorot_uniform(self.num_inputs, self.num_units, rng) if W is None else W
        self.W = nn.Parameter(_as_tensor(w, (self.num_inputs, self.num_units), self.device))
        if b is None:
            self.b = None
        else:
            bb = np.full(self.num_units, float(b), np.float32) if np.isscalar(b) else b
            self.b = nn.Parameter(_as_tensor(bb, (self.num_units,), self.device))
        self.fused_act, self.post = _resolve_nonlinearity(nonlinearity)
        self.mode = mode
        self._cache = {}

    def forward(self, input, **kwargs):
        if not (isinstance(input, gs.DeviceCSR) or sps.issparse(input)):
            raise ValueError("Input for this layer must be sparse")
        X = _upload_cached(self._cache, input, self.device)
        Y = csr_matmul(X, self.W, self.b, self.fused_act, None, self.mode)
        return self.post(Y) if self.post is not None else Y

    def get_output_for(self, input, **kwargs):
        return self.forward(input, **kwargs)


class GCN(nn.Module):
    """The 2-layer model MLPCONV.fit builds (mlpconv.py:196-217), inputs resident in HBM.

    forward(target_indices) -> softmax probabilities of the target rows.
    """

    def __init__(self, H, X, in_features: int, hidden: int, n_classes: int,
                 device="cuda", W1=None, W2=None, mode: str = "auto", rng=None):
        super().__init__()
        self.device = torch.device(device)
        Hd = _as_device_csr(H, self.device)  # symmetry checked at the first backward
        self.X = _as_device_csr(X, self.device)
        if isinstance(rng, (int, np.integer)):
            # one stream for both layers: W1 then W2 drawn in sequence (an int handed to each
            # layer separately would restart the stream and make W2 a rescaled copy of W1)
            rng = np.random.RandomState(int(rng))
        self.l_hid1 = SparseConvolutionDenseLayer(in_features, H=Hd, num_units=hidden, W=W1,
                                                  nonlinearity="rectify", device=self.device,
                                                  mode=mode, rng=rng)
        self.l_out = ConvolutionDenseLayer(self.l_hid1, H=self.l_hid1.H, num_units=n_classes,
                                           W=W2, nonlinearity="softmax", device=self.device,
                                           mode=mode, rng=rng)

    def forward(self, target_indices):
        h = self.l_hid1(self.X)
        return self.l_out(h, target_indices=target_indices)
