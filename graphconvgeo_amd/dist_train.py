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
  backward  the gradient of Y_p = H_p . Z w.r.t. Z, reduced to rank p's rows, is
            (H^T)_p . exchange(g): for a symmetric H (checked once on the host,
            distributed.host_is_symmetric) that is H_p -- the same exchange and the same local
            SpMM as the forward; any other H (the row-normalized D^-1 (A+I) of main.py:451-455)
            gets a second partition of CSR(H^T) over the same row bounds, Theano's H^T . gz.
            dW1 = X_p^T . dZ1_p, dW2, db local.
  all-reduce  ONE bucket with every parameter gradient (W1: F x K = 60 MB at Twitter-World,
            W2 1.1 MB, the biases) over RCCL, then the replicated Lasagne-Adam update.

Per-row arithmetic is unchanged by the partition (every H_p row keeps its storage order), so
the activations and the local gradient rows are bitwise those of the single-GPU step; the
weight gradients differ only by the order of the cross-rank sum.
"""
from __future__ import annotations

import logging
import math
from typing import Optional

import numpy as np
import scipy.sparse as sps
import torch
import torch.distributed as dist

from . import dense
from . import sparse as gs
from .distributed import (RowPartitionedCSR, TargetRows, host_is_symmetric,  # noqa: F401
                          local_targets)
from .layers import _glorot_uniform, csr_matmul
from .mlpconv import LasagneAdam, trainer_order

log = logging.getLogger(__name__)


class GPUOps:
    """Rank-local kernels of the partitioned propagate (HIP). Tests inject CPU versions."""

    @staticmethod
    def empty(n: int, K: int, device) -> torch.Tensor:
        return gs.empty_dense(n, K, device)

    @staticmethod
    def empty_gate(n: int, K: int, device) -> torch.Tensor:
        return gs.empty_gate(n, K, device)

    @staticmethod
    def spmm_into(A, Z, out, bias=None, act=None, rows=None, gate=None, mode="auto"):
        """out = act(A . Z + bias)[rows] (sparse.spmm), the rectify gate bytes into `gate`."""
        return gs.spmm(A, Z, bias=bias, act=act, rows=rows, mode=mode, out=out, gate=gate)

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
        """out[rows[i]] += g[i] into n_rows zero rows, duplicates added in increasing i."""
        from .layers import _index_csr_cached
        full = torch.zeros((n_rows, g.shape[1]), dtype=torch.float32, device=g.device)
        if rows.n:
            seg_ptr, pos = _index_csr_cached(rows, n_rows)
            gs.scatter_add_rows(full, seg_ptr, pos, g.contiguous())
        return full


class _PartitionedPropagate(torch.autograd.Function):
    """Y_p = act(H_p . exchange(Z_p) + b)[targets_p], the exchange pipelined with the SpMM over
    column chunks (distributed.pipelined_product). Backward through part_bwd, the partition of
    H^T over the same row bounds (part itself when H is symmetric):
      no targets: dZ_p = (H^T)_p . exchange(g . act')
      targets   : dZ_p = (H^T)_p[:, D] . exchange(g_D)       (TargetRowsBackward: only the
                  distinct targets' gradient rows travel, only their columns are multiplied)"""

    @staticmethod
    def forward(ctx, Z_p, bias, part: RowPartitionedCSR, act, targets, mode, ops, part_bwd):
        K = Z_p.shape[1]
        rows = None if targets is None else targets.rows
        n_out = part.n_local if rows is None else rows.n
        b = None if bias is None else bias.detach()
        gate = None
        if act == "relu" and any(ctx.needs_input_grad[:2]):
            gate = ops.empty_gate(n_out, K, part.device)
        Y = ops.empty(n_out, K, part.device)

        def into(A, Z, out, **kw):
            return ops.spmm_into(A, Z, out, **kw)
        part.spmm_pipelined(Z_p.detach(), Y, bias=b, gate=gate, act=act, rows=rows, mode=mode,
                            spmm_into=into)
        ctx.part, ctx.act, ctx.targets, ctx.mode, ctx.ops = part, act, targets, mode, ops
        ctx.part_bwd = part if part_bwd is None else part_bwd
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
            part, ops = ctx.part_bwd, ctx.ops
            g = g.contiguous()
            if ctx.targets is not None:
                g_Z = part.target_backward(ctx.targets).backward(g, ops, mode=ctx.mode)
            else:
                g_Z = ops.empty(part.n_local, g.shape[1], part.device)

                def into(A, Z, out, **kw):
                    return ops.spmm_into(A, Z, out, **kw)
                part.spmm_pipelined(g, g_Z, mode=ctx.mode, spmm_into=into)
            if g_Z.shape[0] != ctx.n_in:  # Z_p was given padded to block_rows (all-gather)
                pad = torch.zeros((ctx.n_in, g_Z.shape[1]), dtype=g_Z.dtype, device=g_Z.device)
                pad[: g_Z.shape[0]] = g_Z
                g_Z = pad
        return g_Z, g_bias, None, None, None, None, None, None


def partitioned_propagate(Z_p, part, bias=None, act=None, targets=None, mode="auto", ops=GPUOps,
                          part_bwd=None):
    """Differentiable (H . Z + b)[targets] restricted to rank p's rows, Z row-partitioned;
    targets: None (every local row) or a distributed.TargetRows. part_bwd: the partition of
    H^T over part's row bounds for the backward (None: H is symmetric, part serves both)."""
    if targets is not None and not isinstance(targets, TargetRows):
        raise TypeError("targets must be a distributed.TargetRows (every rank's target list)")
    if part_bwd is not None and not np.array_equal(part_bwd.bounds, part.bounds):
        raise ValueError("part_bwd must partition H^T over the same row bounds as part")
    return _PartitionedPropagate.apply(Z_p, bias, part, act, targets, mode, ops, part_bwd)


class PartitionTargets(TargetRows):
    """One target list (train / dev / test indices, the reference's `target_indices`) split
    over the row partition: rank p keeps the targets in its rows [start, stop), in original
    order. Default: `rows` are the distinct local rows (increasing) with `weight` their
    multiplicities (None when no row repeats) and `y` the label of each distinct row (from
    y_all, the labels of every node); `inverse` maps every kept target to its distinct row, `pos`
    every kept target to its place in the global list. With y_targets (one label per target of
    the global list, e.g. accuracy's y_true): every kept target is its own row, with its own
    label -- duplicates may then disagree (MLPCONV.accuracy compares each target with its own)."""

    def __init__(self, idx, y_all, part: RowPartitionedCSR, device=None, y_targets=None):
        distinct = y_targets is None
        super().__init__(idx, part, distinct=distinct)
        device = part.device if device is None else device
        n_kept = int(self.pos.size)
        if distinct:
            self.inverse = torch.as_tensor(self.inverse_host.astype(np.int64), device=device)
            self.weight = None if self.counts.size == n_kept else \
                torch.as_tensor(self.counts.astype(np.float32), device=device)
            self.y = None if y_all is None else torch.as_tensor(
                np.asarray(y_all)[self.idx[self.pos][self.first]].astype(np.int32), device=device)
        else:
            self.inverse = torch.arange(n_kept, dtype=torch.int64, device=device)
            self.weight = None
            y_t = np.asarray(y_targets)
            if y_t.shape != self.idx.shape:
                raise ValueError("y_targets must hold one label per target")
            self.y = torch.as_tensor(y_t[self.pos].astype(np.int32), device=device)


class RowPartitionedGCN:
    """The MLPCONV network (mlpconv.py:196-217) trained with a 1-D row partition.

    Every rank passes the same host H (the normalized operator), X, train indices and labels
    (each rank keeps only its block); parameters are initialised identically (explicit W1/W2
    or a shared seed) and broadcast from rank 0. Further target lists (dev, test) are added
    with add_targets(); loss / accuracy / probabilities are per named list.
    """

    def __init__(self, H, X, train_indices, y, hidden: int, n_classes: int, rank: int,
                 world: int, device, W1=None, W2=None, order: str = "propagate_first",
                 exchange: str = "auto", mode: str = "auto", regul_coefs=(5e-5, 5e-5),
                 seed: int = 77, group=None, rng=None, symmetric: Optional[bool] = None):
        if order not in ("reference", "propagate_first"):
            raise ValueError("order must be 'reference' or 'propagate_first'")
        self.rank, self.world, self.group = rank, world, group
        self.device = torch.device(device)
        self.order, self.mode = order, mode
        self.regul_coefs = tuple(regul_coefs)
        H = sps.csr_matrix(H)
        self.part = RowPartitionedCSR(H, rank, world, self.device, group=group, exchange=exchange)
        # the backward's operator H^T (Theano's S.dot gradient, mlpconv.py:73,90): H_p itself
        # for a symmetric H, else a partition of CSR(H^T) over the same row bounds. Every rank
        # decides from the same host H, so all take the same branch.
        self.symmetric = host_is_symmetric(H) if symmetric is None else bool(symmetric)
        self.part_t = None if self.symmetric else RowPartitionedCSR(
            H.T.tocsr(), rank, world, self.device, group=group, exchange=self.part.exchange,
            bounds=self.part.bounds)
        self.mode = self.part.resolve_mode(mode)  # one SpMM mode on every rank (the whole graph's)
        start, stop = self.part.start, self.part.stop
        Xc = sps.csr_matrix(X)[start:stop]
        self.X_p = gs.DeviceCSR.from_scipy(Xc, self.device)
        self.n_classes = int(n_classes)
        self._y_all = np.asarray(y)
        self.targets = {}
        self.add_targets("train", train_indices)
        F = X.shape[1]
        # every rank draws the same W1, W2 (then broadcast); rng: a shared RandomState / seed
        rng = np.random.RandomState(seed) if rng is None else rng
        w1 = torch.as_tensor(_glorot_uniform(F, hidden, rng) if W1 is None else np.asarray(W1))
        w2 = torch.as_tensor(_glorot_uniform(hidden, n_classes, rng) if W2 is None
                             else np.asarray(W2))
        self.W1 = torch.nn.Parameter(w1.to(self.device, torch.float32).contiguous())
        self.b1 = torch.nn.Parameter(torch.zeros(hidden, device=self.device))
        self.W2 = torch.nn.Parameter(w2.to(self.device, torch.float32).contiguous())
        self.b2 = torch.nn.Parameter(torch.zeros(n_classes, device=self.device))
        self.params = [self.W1, self.b1, self.W2, self.b2]
        if world > 1:
            self.broadcast_params()
        self.proj = dense.Projection()
        sizes = [p.numel() for p in self.params]
        self._bucket = torch.empty(sum(sizes), dtype=torch.float32, device=self.device)
        self._sizes = sizes

    def add_targets(self, name: str, idx, y=None, y_targets=None):
        """Register a target list (the reference's dev / test indices) under `name`; labels from
        the y given at construction unless `y` (labels of every node) or `y_targets` (one label
        per target, duplicates may differ) is passed."""
        self.targets[name] = PartitionTargets(idx, self._y_all if y is None else y, self.part,
                                              self.device, y_targets=y_targets)

    @torch.no_grad()
    def broadcast_params(self):
        for p in self.params:
            dist.broadcast(p.data, src=0, group=self.group)

    # back-compat views of the training list
    @property
    def rows(self):
        return self.targets["train"].rows

    @property
    def T_total(self):
        return self.targets["train"].total

    # -- forward ------------------------------------------------------------------------
    def _hidden(self):
        Z1 = csr_matmul(self.X_p, self.W1, mode=self.mode)  # S.dot(X_p, W1), mlpconv.py:71
        return partitioned_propagate(Z1, self.part, self.b1, "relu", None, self.mode,
                                     part_bwd=self.part_t)

    def local_loss_acc(self, name: str = "train", penalty: bool = True):
        """This rank's share of (mean CE + penalty, accuracy) over all ranks' targets of the
        list `name` (the mean is over the whole list; the penalty is counted on rank 0)."""
        tg = self.targets[name]
        h = self._hidden()
        if self.order == "propagate_first":
            P = partitioned_propagate(h, self.part, None, None, tg, self.mode, part_bwd=self.part_t)
            loss, acc = self.proj.softmax_xent(P, self.W2, self.b2, tg.y, denom=tg.total,
                                               row_weight=tg.weight)
        else:
            Z2 = dense.matmul(h, self.W2)  # T.dot(h, W2), mlpconv.py:88
            logits = partitioned_propagate(Z2, self.part, self.b2, None, tg, self.mode,
                                            part_bwd=self.part_t)
            loss, acc = dense.softmax_xent(logits, tg.y, denom=tg.total, row_weight=tg.weight)
        if penalty and self.rank == 0:
            c_out, c_hid = self.regul_coefs  # mlpconv.py:235-243, counted once
            loss = loss + dense.l1l2_penalty([self.W2, self.W1], [(c_out * 0.5, c_out * 0.5),
                                                                   (c_hid * 0.5, c_hid * 0.5)])
        return loss, acc

    def _allreduce(self, t: torch.Tensor) -> torch.Tensor:
        if self.world > 1:
            dist.all_reduce(t, group=self.group)
        return t

    @torch.no_grad()
    def evaluate(self, name: str, penalty: bool = True):
        """Global (loss, acc) of the list `name` (forward only, all-reduced), as device scalars."""
        loss, acc = self.local_loss_acc(name, penalty=penalty)
        stats = self._allreduce(torch.stack([loss.detach().reshape(()), acc.detach().reshape(())]))
        return stats[0], stats[1]

    @torch.no_grad()
    def local_probabilities(self, name: str) -> torch.Tensor:
        """softmax rows of this rank's kept targets of `name`, in their global order."""
        tg = self.targets[name]
        h = self._hidden()
        if self.order == "propagate_first" and self.n_classes <= dense.FUSED_MAX_COLS:
            P = partitioned_propagate(h, self.part, None, None, tg, self.mode, part_bwd=self.part_t)
            probs = self.proj.probabilities(P, self.W2, self.b2)
        else:
            if self.order == "propagate_first":
                P = partitioned_propagate(h, self.part, None, None, tg, self.mode,
                                          part_bwd=self.part_t)
                logits = dense.matmul(P, self.W2, self.b2)
            else:
                Z2 = dense.matmul(h, self.W2)
                logits = partitioned_propagate(Z2, self.part, self.b2, None, tg, self.mode,
                                            part_bwd=self.part_t)
            probs = dense.softmax(logits)
        return probs.index_select(0, tg.inverse)

    @torch.no_grad()
    def gather_probabilities(self, name: str, dst: int = 0):
        """The whole list's probabilities [T, C] (original target order) on rank `dst` only
        (None elsewhere): each rank sends its kept rows, padded to the largest share."""
        tg = self.targets[name]
        local = self.local_probabilities(name).contiguous()
        if self.world == 1:
            return local.cpu().numpy()
        b = self.part.bounds
        shares = [local_targets(tg.idx, int(b[q]), int(b[q + 1]))[0] for q in range(self.world)]
        m = max(max(x.size for x in shares), 1)
        send = torch.zeros((m, self.n_classes), dtype=torch.float32, device=self.device)
        send[: len(tg)] = local
        recv = [torch.empty_like(send) for _ in range(self.world)] if self.rank == dst else None
        dist.gather(send, recv, dst=dst, group=self.group)
        if self.rank != dst:
            return None
        out = np.empty((tg.total, self.n_classes), dtype=np.float32)
        for q, pos in enumerate(shares):
            out[pos] = recv[q][: pos.size].cpu().numpy()
        return out

    # -- one optimisation step -----------------------------------------------------------
    def allreduce_grads(self):
        """One bucketed all-reduce (sum) of every parameter gradient."""
        off = 0
        for p, n in zip(self.params, self._sizes):
            self._bucket[off:off + n].copy_(p.grad.reshape(-1))
            off += n
        self._allreduce(self._bucket)
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
        stats = self._allreduce(torch.stack([loss.detach(), acc.detach()]))
        return stats[0], stats[1]

    def make_optimizer(self, lr=4e-3) -> LasagneAdam:
        return LasagneAdam(self.params, lr=lr, beta1=0.9, beta2=0.999, epsilon=1e-8)


class RowPartitionedMLPCONV:
    """MLPCONV.fit / predict / predict_proba / accuracy / score (mlpconv.py:152-349) over a
    1-D row partition: one process per GPU, every rank calls the same methods with the same
    host arguments (each keeps its block). Same constructor arguments as MLPCONV plus
    rank / world / group / exchange; the epoch loop, validation every report_k_epoch,
    best-parameter restore, early stopping and the final dev evaluation follow MLPCONV.fit
    (graphconvgeo_amd/mlpconv.py), with every loss and hit count all-reduced so that every rank
    takes the same decisions. predict / predict_proba return the requested partition's rows on
    rank 0 (None on the other ranks); accuracy and score are global on every rank."""

    def __init__(self, n_epochs=10, batch_size=1000, init_parameters=None, complete_prob=False,
                 add_hidden=True, regul_coefs=(5e-5, 5e-5), save_results=False,
                 hidden_layer_size=None, drop_out=False, dropout_coefs=(0.5, 0.5),
                 early_stopping_max_down=100000, loss_name="log", nonlinearity="rectify",
                 dtype="float32", device="cuda", seed: Optional[int] = None, mode: str = "auto",
                 model_file: Optional[str] = None, report_k_epoch: int = 10,
                 order: str = "auto", rank: Optional[int] = None,
                 world: Optional[int] = None, group=None, exchange: str = "auto",
                 network_factory=None):
        if dtype != "float32":
            raise ValueError("the GPU path computes in float32 (mlpconv.py dtype='float32')")
        if drop_out:
            raise NotImplementedError("dropout is out of scope (main_mlpconv uses drop_out=False)")
        if complete_prob:
            raise NotImplementedError("complete_prob (soft labels) is not on the graded path")
        if loss_name != "log":
            raise ValueError("only the 'log' (categorical cross-entropy) loss exists in the reference")
        if order not in ("reference", "propagate_first", "auto"):
            raise ValueError("order must be 'reference', 'propagate_first' or 'auto'")
        self.n_epochs = n_epochs
        self.batch_size = batch_size
        self.init_parameters = init_parameters
        self.regul_coefs = list(regul_coefs)
        self.hidden_layer_size = hidden_layer_size
        self.dropout_coefs = list(dropout_coefs)
        self.early_stopping_max_down = early_stopping_max_down
        self.device = torch.device(device)
        self.seed, self.mode, self.order = seed, mode, order
        self.model_file = model_file
        self.report_k_epoch = report_k_epoch
        self.rank = dist.get_rank(group) if rank is None else rank
        self.world = dist.get_world_size(group) if world is None else world
        self.group, self.exchange = group, exchange
        self.network_factory = network_factory or RowPartitionedGCN
        self.history = []

    def fit(self, X, train_indices, dev_indices, test_indices, Y, H):
        """mlpconv.py:152-318 over the row partition (full-batch epochs)."""
        Y = np.asarray(Y)
        if Y.ndim != 1 or not np.issubdtype(Y.dtype, np.integer):
            raise ValueError("Y must be a 1-D integer label array (complete_prob is out of scope)")
        if Y.size and int(Y.min()) < 0:
            raise ValueError("labels must be >= 0 (class ids, data.py:399-432)")
        if self.hidden_layer_size is None:
            raise ValueError("hidden_layer_size is required")
        out_size = int(np.max(Y)) + 1
        order = trainer_order(self.order, self.hidden_layer_size, out_size)  # as MLPCONV
        W1 = W2 = None
        if self.init_parameters is not None:
            W1, _b1, W2, _b2 = self.init_parameters
        # Lasagne GlorotUniform from numpy's global stream (W1 then W2) unless a seed is given;
        # every rank draws, rank 0's draw is broadcast
        rng = np.random.mtrand._rand if self.seed is None else np.random.RandomState(self.seed)
        idx = {"train": np.asarray(train_indices, np.int32), "dev": np.asarray(dev_indices, np.int32),
               "test": np.asarray(test_indices, np.int32)}
        net = self.network_factory(H, X, idx["train"], Y, hidden=self.hidden_layer_size,
                                   n_classes=out_size, rank=self.rank, world=self.world,
                                   device=self.device, W1=W1, W2=W2, order=order,
                                   exchange=self.exchange, mode=self.mode,
                                   regul_coefs=self.regul_coefs, group=self.group, rng=rng)
        for k in ("dev", "test"):
            net.add_targets(k, idx[k])
        if self.init_parameters is not None:
            with torch.no_grad():
                net.b1.copy_(torch.as_tensor(self.init_parameters[1]))
                net.b2.copy_(torch.as_tensor(self.init_parameters[3]))
        self.net = net
        self.params = net.params
        opt = net.make_optimizer()
        self.optimizer = opt
        best_params, best_val_loss, best_val_acc, n_down = None, math.inf, 0.0, 0
        for n in range(self.n_epochs):
            loss, acc = net.train_step(opt)
            rec = {"epoch": n, "train_loss": float(loss), "train_acc": float(acc)}
            if n % self.report_k_epoch == 0:
                l_val, a_val = (float(x) for x in net.evaluate("dev"))
                rec.update(val_loss=l_val, val_acc=a_val)
                if l_val < best_val_loss:
                    best_val_loss, best_val_acc, n_down = l_val, a_val, 0
                    best_params = [p.detach().clone() for p in self.params]
                else:
                    n_down += 1
                log.info("epoch %d ,train_loss %s ,acc %s ,val_loss %s ,acc %s,best_val_acc %s",
                         n, rec["train_loss"], rec["train_acc"], l_val, a_val, best_val_acc)
                self.history.append(rec)
                if n_down > self.early_stopping_max_down:
                    log.info("validation results went down. early stopping ...")
                    break
            else:
                self.history.append(rec)
        if best_params is not None:
            with torch.no_grad():
                for p, b in zip(self.params, best_params):
                    p.copy_(b)
        if self.model_file and self.rank == 0:
            torch.save([p.detach().cpu() for p in self.params], self.model_file)
            self.model_path = self.model_file
        l_val, a_val = net.evaluate("dev")  # final dev evaluation, mlpconv.py:316-318
        self.best_dev_loss, self.best_dev_acc = float(l_val), float(a_val)
        log.info("Best dev acc: %f", self.best_dev_acc)
        return self

    def _check(self, partition):
        if partition not in ("train", "dev", "test"):
            raise ValueError(f"unknown partition {partition!r}")

    def predict_proba(self, dataset_partition):
        self._check(dataset_partition)
        return self.net.gather_probabilities(dataset_partition, dst=0)

    def predict(self, dataset_partition):
        proba = self.predict_proba(dataset_partition)
        return None if proba is None else proba.argmax(axis=1)

    def accuracy(self, dataset_partition, y_true):
        """Global accuracy of the partition against y_true (the labels of its targets, in
        target order), on every rank."""
        self._check(dataset_partition)
        idx = self.net.targets[dataset_partition].idx
        y_true = np.asarray(y_true)
        if y_true.shape != idx.shape:
            raise ValueError("y_true must hold one label per target of the partition")
        # one label per target (duplicates drawn with replacement may carry different labels:
        # each is scored against its own, as MLPCONV.accuracy does)
        self.net.add_targets("_accuracy", idx, y_targets=y_true)
        try:
            _loss, acc = self.net.evaluate("_accuracy", penalty=False)
        finally:
            del self.net.targets["_accuracy"]
        return float(acc)

    def score(self, X, dataset_partition, y_true):
        """mlpconv.py:348-349 signature (see MLPCONV.score)."""
        return self.accuracy(dataset_partition, y_true)

    def get_params(self):
        return [p.detach().cpu().numpy() for p in self.params]


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
