"""Row-partitioned GCN training step across the GPUs of one node.

The reference trains single-process (MLPCONV.fit, mlpconv.py:152-318). Here rank p owns a
contiguous nnz-balanced block of rows of H, of X and of every N-row activation; the weights
W1, b1, W2, b2 are replicated. Per step:

  forward   Z1_p = X_p . W1                                      local SpMM, no exchange
            h_p  = rectify(H_p . exchange(Z1_p) + b1)             exchange = all-gather / halo
            order "propagate_first":
              P_p = (H_p . exchange(h_p))[targets_p]              K wide
              loss_p, hits_p, G_p = fused MFMA output layer       (dense.py)
            order "reference":
              logits_p = (H_p . exchange(h_p . W2) + b2)[targets_p]   C wide
              loss_p, hits_p = softmax-CE row kernel
            the mean is over ALL ranks' targets (1/T_total), the penalty is added on rank 0
  backward  through H's symmetry: the gradient of Y_p = H_p . Z w.r.t. Z, reduced to rank p's
            rows, is H_p . exchange(g) -- the same exchange and the same local SpMM as the
            forward (H^T = H, so row block p of H^T is H_p). dW1 = X_p^T . dZ1_p, dW2, db local.
  all-reduce  ONE bucket with every parameter gradient (W1: F x K = 60 MB at Twitter-World,
            W2 1.1 MB, the biases) over RCCL, then the replicated Lasagne-Adam update.

Per-row arithmetic is unchanged by the partition (every H_p row keeps its storage order), so
the activations and the local gradient rows are bitwise those of the single-GPU step; the
weight gradients differ only by the order of the cross-rank sum.
"""
from __future__ import annotations

import math
from typing import Optional

import numpy as np
import scipy.sparse as sps
import torch
import torch.distributed as dist

from . import dense
from . import sparse as gs
from .distributed import RowPartitionedCSR
from .layers import _glorot_uniform, csr_matmul
from .mlpconv import LasagneAdam


class GPUOps:
    """Rank-local kernels of the partitioned propagate (HIP). Tests inject CPU versions."""

    @staticmethod
    def spmm(A, Z, bias=None, act=None, rows=None, mode="auto", want_gate=False):
        """Y, or (Y, gate) with the rectify gate bytes (sparse.spmm(gate=...)) if want_gate."""
        if not want_gate:
            return gs.spmm(A, Z, bias=bias, act=act, rows=rows, mode=mode)
        n_out = A.n_rows if rows is None else len(rows)
        gate = gs.empty_gate(n_out, Z.shape[1], A.device)
        return gs.spmm(A, Z, bias=bias, act=act, rows=rows, mode=mode, gate=gate), gate

    @staticmethod
    def relu_backward(gY, gate, bias_grad=True):
        """Theano's rectify gradient (g, g/2, 0 for gate 2, 1, 0) + the bias gradient."""
        if gY.shape[1] <= 1024:
            return gs.relu_backward(gY if gY.stride(-1) == 1 else gY.contiguous(), gate=gate,
                                    bias_grad=bias_grad)
        g = gY * (gate.to(gY.dtype) * 0.5)
        return g, (g.sum(dim=0) if bias_grad else None)

    @staticmethod
    def scatter_rows(n_rows: int, rows: gs.RowSelection, g: torch.Tensor) -> torch.Tensor:
        from .layers import _index_csr_cached
        full = torch.zeros((n_rows, g.shape[1]), dtype=torch.float32, device=g.device)
        if rows.n:
            seg_ptr, pos = _index_csr_cached(rows, n_rows)
            gs.scatter_add_rows(full, seg_ptr, pos, g.contiguous())
        return full


class _PartitionedPropagate(torch.autograd.Function):
    """Y_p = act(H_p . exchange(Z_p) + b)[rows_p]; dZ_p = H_p . exchange(scatter(g . act'))."""

    @staticmethod
    def forward(ctx, Z_p, bias, part: RowPartitionedCSR, act, rows, mode, ops):
        operand = part.all_gather(Z_p.detach())
        b = None if bias is None else bias.detach()
        gate = None
        if act == "relu" and any(ctx.needs_input_grad[:2]):
            Y, gate = ops.spmm(part.A, operand, bias=b, act=act, rows=rows, mode=mode,
                               want_gate=True)
        else:
            Y = ops.spmm(part.A, operand, bias=b, act=act, rows=rows, mode=mode)
        ctx.part, ctx.act, ctx.rows, ctx.mode, ctx.ops = part, act, rows, mode, ops
        ctx.has_bias = bias is not None
        ctx.n_in = Z_p.shape[0]
        ctx.save_for_backward(gate)
        return Y

    @staticmethod
    def backward(ctx, gY):
        (gate,) = ctx.saved_tensors
        want_bias = ctx.has_bias and ctx.needs_input_grad[1]
        if gate is None:
            g, g_bias = gY, (gY.sum(dim=0) if want_bias else None)
        else:
            g, g_bias = ctx.ops.relu_backward(gY, gate, bias_grad=want_bias)
        g_Z = None
        if ctx.needs_input_grad[0]:
            part = ctx.part
            if ctx.rows is not None:
                g = ctx.ops.scatter_rows(part.n_local, ctx.rows, g)
            operand = part.all_gather(g.contiguous())
            g_Z = ctx.ops.spmm(part.A, operand, mode=ctx.mode)
            if g_Z.shape[0] != ctx.n_in:  # Z_p was given padded to block_rows (all-gather)
                pad = torch.zeros((ctx.n_in, g_Z.shape[1]), dtype=g_Z.dtype, device=g_Z.device)
                pad[: g_Z.shape[0]] = g_Z
                g_Z = pad
        return g_Z, g_bias, None, None, None, None, None


def partitioned_propagate(Z_p, part, bias=None, act=None, rows=None, mode="auto", ops=GPUOps):
    """Differentiable (H . Z + b)[rows] restricted to rank p's rows, Z row-partitioned."""
    return _PartitionedPropagate.apply(Z_p, bias, part, act, rows, mode, ops)


def local_targets(idx: np.ndarray, start: int, stop: int):
    """Positions and local row ids of the targets that fall in [start, stop), original order."""
    idx = np.asarray(idx)
    pos = np.nonzero((idx >= start) & (idx < stop))[0]
    return pos, (idx[pos] - start).astype(np.int32)


class RowPartitionedGCN:
    """The MLPCONV network (mlpconv.py:196-217) trained with a 1-D row partition.

    Every rank passes the same host H (the normalized operator), X, train indices and labels
    (each rank keeps only its block); parameters are initialised identically (explicit W1/W2
    or a shared seed) and broadcast from rank 0.
    """

    def __init__(self, H, X, train_indices, y, hidden: int, n_classes: int, rank: int,
                 world: int, device, W1=None, W2=None, order: str = "propagate_first",
                 exchange: str = "auto", mode: str = "auto", regul_coefs=(5e-5, 5e-5),
                 seed: int = 77, group=None):
        if order not in ("reference", "propagate_first"):
            raise ValueError("order must be 'reference' or 'propagate_first'")
        self.rank, self.world, self.group = rank, world, group
        self.device = torch.device(device)
        self.order, self.mode = order, mode
        self.regul_coefs = tuple(regul_coefs)
        H = sps.csr_matrix(H)
        self.part = RowPartitionedCSR(H, rank, world, self.device, group=group, exchange=exchange)
        start, stop = self.part.start, self.part.stop
        Xc = sps.csr_matrix(X)[start:stop]
        self.X_p = gs.DeviceCSR.from_scipy(Xc, self.device)
        idx = np.asarray(train_indices)
        self.T_total = int(idx.size)
        pos, loc = local_targets(idx, start, stop)
        self.rows = gs.RowSelection(loc, self.device)
        self.y_p = torch.as_tensor(np.asarray(y)[idx[pos]].astype(np.int32), device=self.device)
        # repeated local targets (drawn with replacement): the output layer runs on the
        # distinct rows, weighted by multiplicity (MLPCONV._loss_acc does the same)
        self.row_w = None
        d = self.rows.distinct()
        if d is not None:
            self.rows, first, self.row_w = d
            self.y_p = self.y_p.index_select(0, first)
        F = X.shape[1]
        rng = np.random.RandomState(seed)  # every rank draws the same W1, W2 (then broadcast)
        w1 = torch.as_tensor(_glorot_uniform(F, hidden, rng) if W1 is None else np.asarray(W1))
        w2 = torch.as_tensor(_glorot_uniform(hidden, n_classes, rng) if W2 is None
                             else np.asarray(W2))
        self.W1 = torch.nn.Parameter(w1.to(self.device, torch.float32).contiguous())
        self.b1 = torch.nn.Parameter(torch.zeros(hidden, device=self.device))
        self.W2 = torch.nn.Parameter(w2.to(self.device, torch.float32).contiguous())
        self.b2 = torch.nn.Parameter(torch.zeros(n_classes, device=self.device))
        self.params = [self.W1, self.b1, self.W2, self.b2]
        if world > 1:
            with torch.no_grad():
                for p in self.params:
                    dist.broadcast(p.data, src=0, group=group)
        self.proj = dense.Projection()
        sizes = [p.numel() for p in self.params]
        self._bucket = torch.empty(sum(sizes), dtype=torch.float32, device=self.device)
        self._sizes = sizes

    # -- forward ------------------------------------------------------------------------
    def local_loss_acc(self):
        """This rank's share of (mean CE + penalty, accuracy) over all ranks' targets."""
        Z1 = csr_matmul(self.X_p, self.W1, mode=self.mode)  # S.dot(X_p, W1), mlpconv.py:71
        h = partitioned_propagate(Z1, self.part, self.b1, "relu", None, self.mode)
        if self.order == "propagate_first":
            P = partitioned_propagate(h, self.part, None, None, self.rows, self.mode)
            loss, acc = self.proj.softmax_xent(P, self.W2, self.b2, self.y_p, denom=self.T_total,
                                               row_weight=self.row_w)
        else:
            Z2 = dense.matmul(h, self.W2)  # T.dot(h, W2), mlpconv.py:88
            logits = partitioned_propagate(Z2, self.part, self.b2, None, self.rows, self.mode)
            loss, acc = dense.softmax_xent(logits, self.y_p, denom=self.T_total,
                                           row_weight=self.row_w)
        if self.rank == 0:
            c_out, c_hid = self.regul_coefs  # mlpconv.py:235-243, counted once
            loss = loss + dense.l1l2_penalty([self.W2, self.W1], [(c_out * 0.5, c_out * 0.5),
                                                                   (c_hid * 0.5, c_hid * 0.5)])
        return loss, acc

    # -- one optimisation step -----------------------------------------------------------
    def allreduce_grads(self):
        """One bucketed all-reduce (sum) of every parameter gradient."""
        off = 0
        for p, n in zip(self.params, self._sizes):
            self._bucket[off:off + n].copy_(p.grad.reshape(-1))
            off += n
        if self.world > 1:
            dist.all_reduce(self._bucket, group=self.group)
        off = 0
        for p, n in zip(self.params, self._sizes):
            p.grad.copy_(self._bucket[off:off + n].view_as(p.grad))
            off += n

    def train_step(self, opt: LasagneAdam):
        """fwd + bwd + all-reduce + Adam. Returns the global (loss, acc) as device scalars."""
        opt.zero_grad()
        loss, acc = self.local_loss_acc()
        loss.backward()
        for p in self.params:
            if p.grad is None:
                p.grad = torch.zeros_like(p)
        self.allreduce_grads()
        opt.step()
        stats = torch.stack([loss.detach(), acc.detach()])
        if self.world > 1:
            dist.all_reduce(stats, group=self.group)
        return stats[0], stats[1]

    def make_optimizer(self, lr=4e-3) -> LasagneAdam:
        return LasagneAdam(self.params, lr=lr, beta1=0.9, beta2=0.999, epsilon=1e-8)


def spmm_bytes_per_step(part: RowPartitionedCSR, X_p: gs.DeviceCSR, K: int, n_targets: int,
                        order: str, C: int) -> int:
    """Edge-centric algorithmic bytes of this rank's SpMMs in one step (reporting)."""
    def b(n_out, nnz, k):
        return 4 * (n_out + 1) + 8 * nnz + 4 * k * nnz + 4 * k * n_out
    nl, nnz = part.n_local, part.nnz_local
    tot = b(nl, X_p.nnz, K) * 2 + b(nl, nnz, K) * 2  # X.W1, X^T.dZ1, H.Z1 and its backward
    frac = n_targets / max(nl, 1)
    w = K if order == "propagate_first" else C
    tot += b(n_targets, int(nnz * min(frac, 1.0)), w) + b(nl, nnz, w)
    return tot
