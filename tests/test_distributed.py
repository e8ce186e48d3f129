"""world_size-2 gloo tests of the 1-D row partition on CPU.

The rank-local SpMM is the CPU oracle injected as `local_spmm` (test-only); the
partition, column remap and all-gather logic are the product code the RCCL path runs.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from graphconvgeo_amd.synth import synthetic_graph


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run_world(target, world, *args, results: int = 1, timeout: float = 180):
    """Spawn `world` gloo ranks of target(rank, world, port, *args, q); returns the `results`
    items the ranks put on q. Ranks still alive afterwards (a mismatched collective hangs) are
    killed, so a failing case cannot leave processes behind."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port) + tuple(args) + (q,))
             for r in range(world)]
    for p in procs:
        p.start()
    try:
        out = [q.get(timeout=timeout) for _ in range(results)]
        for p in procs:
            p.join(timeout=60)
            assert p.exitcode == 0
    finally:
        for p in procs:
            if p.is_alive():
                p.kill()
                p.join(timeout=10)
    return out


def _oracle_spmm(A, Z_full, out=None, bias=None, act=None, rows=None, gate=None, **kw):
    """Test-only rank-local SpMM: the CPU oracle with the HIP entry's epilogue arguments."""
    from oracle import gcn_oracle as O
    r = None if rows is None else rows.host
    b = None if bias is None else bias.numpy()
    pre = O.spmm_f32(A, np.ascontiguousarray(Z_full.numpy()), bias=b, rows=r)
    Y = torch.from_numpy(O.relu(pre) if act == "relu" else pre)
    if gate is not None:
        gate.copy_(torch.from_numpy((2 * (pre > 0) + (pre == 0)).astype(np.uint8)))
    if out is not None:
        out.copy_(Y)
        return out
    return Y


def _worker(rank, world, port, n, e, K, exchange, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from graphconvgeo_amd.distributed import RowPartitionedCSR
        H = synthetic_graph(n, e)
        Z = np.random.default_rng(5).standard_normal((n, K)).astype(np.float32)
        part = RowPartitionedCSR(H, rank, world, "cpu", local_spmm=_oracle_spmm, exchange=exchange)
        assert part.exchange == exchange
        Zl = torch.from_numpy(part.local_rows(Z).copy())
        Y = part.spmm(Zl)
        Yp = torch.empty_like(Y)
        part.spmm_pipelined(Zl, Yp, n_chunks=3)  # 24 cols -> chunks of 8
        assert torch.equal(Y, Yp)
        # the producer writes its rows straight into the exchange buffers: no staging copy
        bufs = part.chunk_buffers(K, 2)
        for (c0, c1, _b), own in zip(bufs.chunks, bufs.own_views()):
            own.copy_(Zl[:own.shape[0], c0:c1])
        Yq = torch.empty_like(Y)
        part.spmm_pipelined(None, Yq, n_chunks=2)
        assert torch.equal(Y, Yq)
        # bias + rectify + gate sliced per chunk, 4 chunks of 6 columns
        bias = torch.from_numpy(np.random.default_rng(8).standard_normal(K).astype(np.float32))
        gate = torch.empty((part.n_local, K), dtype=torch.uint8)
        Yr = torch.empty_like(Y)
        part.spmm_pipelined(Zl, Yr, n_chunks=4, bias=bias, act="relu", gate=gate)
        Yr1 = torch.empty_like(Y)
        gate1 = torch.empty_like(gate)
        part.spmm_pipelined(Zl, Yr1, n_chunks=1, bias=bias, act="relu", gate=gate1)
        assert torch.equal(Yr, Yr1) and torch.equal(gate, gate1)
        # the exchange delivers exactly the rows layout.operand_ids() names (the single-process
        # rehearsal, distributed.LOOPBACK, builds operands from it)
        ids = part.layout.operand_ids()
        full = part.all_gather(Zl).numpy()
        ok = ids >= 0
        assert np.array_equal(full[ok], Z[ids[ok]]) and ids.size == part.operand_rows()
        out = [None] * world
        dist.all_gather_object(out, (part.start, part.stop, Y.numpy()))
        if rank == 0:
            q.put(out)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("exchange", ["allgather", "mesh", "halo"])
@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_row_partitioned_spmm_equals_full(world, exchange):
    from oracle import gcn_oracle as O
    n, e, K = 3000, 20000, 24
    (out,) = _run_world(_worker, world, n, e, K, exchange)
    H = synthetic_graph(n, e)
    Z = np.random.default_rng(5).standard_normal((n, K)).astype(np.float32)
    ref = O.spmm_f32(H, Z)
    got = np.zeros_like(ref)
    covered = 0
    for start, stop, Y in out:
        got[start:stop] = Y
        covered += stop - start
    assert covered == n
    # Same per-row storage order -> bitwise equal to the unpartitioned product.
    assert np.array_equal(got, ref)


def test_halo_layout_and_auto_choice():
    from graphconvgeo_amd.distributed import RowPartitionedCSR
    n, e = 3000, 20000
    H = synthetic_graph(n, e)
    Z = np.random.default_rng(1).standard_normal((n, 8)).astype(np.float32)
    parts = [RowPartitionedCSR(H, r, 4, "cpu", local_spmm=_oracle_spmm, exchange="halo")
             for r in range(4)]
    for p in parts:
        # own rows first, then the halo rows of rank 0..3 (sorted global ids)
        b = p.bounds
        assert sum(p.recv_counts) == p.halo_rows and p.recv_counts[p.rank] == 0
        for q in parts:
            assert q.send_counts[p.rank] == p.recv_counts[q.rank]
        cols = np.unique(H.indices[H.indptr[b[p.rank]]:H.indptr[b[p.rank + 1]]])
        halo = cols[(cols < p.start) | (cols >= p.stop)]
        operand = np.concatenate([Z[p.start:p.stop], Z[halo]])
        from oracle import gcn_oracle as O
        assert np.array_equal(O.spmm_f32(p.local_host, operand), O.spmm_f32(H, Z)[p.start:p.stop])
    dense = RowPartitionedCSR(H, 0, 2, "cpu", local_spmm=_oracle_spmm)  # halo ~100% -> allgather
    assert dense.halo_fraction > 0.9 and dense.exchange == "allgather"


def test_feature_parallel_columns_concatenate_to_full():
    from graphconvgeo_amd.distributed import FeatureParallelSpMM, feature_partition
    from oracle import gcn_oracle as O
    assert feature_partition(300, 8)[0] == (0, 40) and feature_partition(300, 8)[-1] == (280, 300)
    assert feature_partition(10, 4) == [(0, 4), (4, 8), (8, 10), (10, 10)]
    H = synthetic_graph(2000, 12000)
    Z = np.random.default_rng(3).standard_normal((2000, 30)).astype(np.float32)
    ref = O.spmm_f32(H, Z)
    parts = []
    for r in range(3):
        fp = FeatureParallelSpMM(H, r, 3, "cpu", 30, local_spmm=_oracle_spmm)
        parts.append(fp.spmm(torch.from_numpy(np.ascontiguousarray(Z[:, fp.c0:fp.c1]))).numpy())
    assert np.array_equal(np.concatenate(parts, axis=1), ref)  # column-local: bitwise


class _CPUOps:
    """Test-only rank-local ops for the partitioned propagate: the CPU oracle."""

    @staticmethod
    def empty(n, K, device):
        return torch.empty((n, K), dtype=torch.float32)

    @staticmethod
    def empty_gate(n, K, device):
        return torch.empty((n, K), dtype=torch.uint8)

    @staticmethod
    def spmm_into(A, Z, out, bias=None, act=None, rows=None, gate=None, mode="auto"):
        return _oracle_spmm(A, Z, out=out, bias=bias, act=act, rows=rows, gate=gate)

    @staticmethod
    def relu_backward(gY, gate, bias_grad=True):
        g = gY * (gate.to(gY.dtype) * 0.5)
        return g, (g.sum(dim=0) if bias_grad else None)

    @staticmethod
    def scatter_rows(n_rows, rows, g):
        from oracle import gcn_oracle as O
        out = np.zeros((n_rows, g.shape[1]), np.float32)
        O.scatter_add_f32(out, rows.host, g.detach().numpy())
        return torch.from_numpy(out)


def _operator(n, e, nonsym):
    """The symmetric D^-1/2 (A+I) D^-1/2, or the reference's row-normalized D^-1 (A+I)
    (main.py:451-456) -- not symmetric."""
    H = synthetic_graph(n, e)
    if nonsym:
        from oracle import gcn_oracle as O
        A = H.copy()
        A.data[:] = 1.0
        H = O.row_normalize_l1(A)
    return H


def _prop_worker(rank, world, port, n, e, K, exchange, hi, nonsym, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from graphconvgeo_amd.dist_train import partitioned_propagate
        from graphconvgeo_amd.distributed import RowPartitionedCSR, TargetRows, host_is_symmetric
        H = _operator(n, e, nonsym)
        assert host_is_symmetric(H) == (not nonsym)
        rng = np.random.default_rng(11)
        Z = rng.standard_normal((n, K)).astype(np.float32)
        b = rng.standard_normal(K).astype(np.float32)
        targets = rng.integers(0, hi, size=n // 2).astype(np.int32)  # duplicates included
        part = RowPartitionedCSR(H, rank, world, "cpu", local_spmm=_oracle_spmm, exchange=exchange)
        part.chunks_override = 3 if world == 3 else None  # the pipelined form in fwd and bwd
        part_t = None
        if nonsym:  # the backward's H^T, partitioned over the same row bounds
            part_t = RowPartitionedCSR(H.T.tocsr(), rank, world, "cpu", local_spmm=_oracle_spmm,
                                       exchange=exchange, bounds=part.bounds)
            part_t.chunks_override = part.chunks_override
        Zp = torch.from_numpy(part.local_rows(Z).copy()).requires_grad_()
        bt = torch.from_numpy(b).requires_grad_()
        h = partitioned_propagate(Zp, part, bt, "relu", None, ops=_CPUOps, part_bwd=part_t)
        tg = TargetRows(targets, part)  # every kept target, duplicates included
        pos = tg.pos
        P = partitioned_propagate(h, part, None, None, tg, ops=_CPUOps, part_bwd=part_t)
        R = torch.from_numpy(rng.standard_normal((targets.size, K)).astype(np.float32))
        (P * R[torch.from_numpy(pos)]).sum().backward()
        bwd = (part_t or part).target_backward(tg)
        # only the distinct targets' rows travel; the operator keeps only their columns
        assert bwd.layout.counts == [d.size for d in tg.block_distinct]
        assert bwd.nnz <= (part_t or part).nnz_local
        assert tg._backward_op is bwd  # cached on the list, not on the partition
        out = [None] * world
        dist.all_gather_object(out, (part.start, part.stop, pos, P.detach().numpy(),
                                     Zp.grad.numpy(), bt.grad.numpy(), len(tg)))
        if rank == 0:
            q.put(out)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("exchange,world,nonsym", [
    ("allgather", 2, False), ("halo", 2, False), ("mesh", 2, False), ("mesh", 3, False),
    ("allgather", 3, False), ("allgather", 4, False), ("halo", 4, False), ("mesh", 4, False),
    ("allgather", 8, False), ("halo", 8, False), ("mesh", 8, False),
    ("allgather", 2, True), ("halo", 3, True), ("mesh", 4, True)])
def test_partitioned_propagate_fwd_bwd(exchange, world, nonsym):
    """Two stacked partitioned propagates (rectify, then a target-row subset with duplicates)
    and their backward through H^T (H itself for the symmetric operator; a partition of CSR(H^T)
    over the same bounds for the reference's row-normalized D^-1 (A+I), main.py:451-456):
    activations and input gradients bitwise equal to the single-process oracle chain; the bias
    gradient (a cross-rank sum) within fp32. At world 4 and 8 the targets lie in the first 40 %
    of the nodes (the reference's train rows come first): the last ranks hold no target,
    contribute no rows to the target exchange, and still receive the others'."""
    from oracle import gcn_oracle as O
    n, e, K = 2500, 16000, 12
    hi = n if world < 4 else int(0.4 * n)
    (out,) = _run_world(_prop_worker, world, n, e, K, exchange, hi, nonsym)
    H = _operator(n, e, nonsym)
    Ht = H.T.tocsr()  # Theano's S.dot gradient H^T . gz (stable transpose: scipy's order)
    rng = np.random.default_rng(11)
    Z = rng.standard_normal((n, K)).astype(np.float32)
    b = rng.standard_normal(K).astype(np.float32)
    targets = rng.integers(0, hi, size=n // 2).astype(np.int32)
    R = rng.standard_normal((targets.size, K)).astype(np.float32)
    h = O.spmm_f32(H, Z, bias=b, act="relu")
    P = O.spmm_f32(H, h, rows=targets)
    g_h = np.zeros((n, K), np.float32)
    O.scatter_add_f32(g_h, targets, R)
    g_h = O.spmm_f32(Ht, g_h)
    g_pre = g_h * (h > 0)
    g_Z = O.spmm_f32(Ht, g_pre.astype(np.float32))
    got_P = np.zeros_like(P)
    got_gZ = np.zeros_like(g_Z)
    g_b = np.zeros(K, np.float64)
    n_targets = []
    for start, stop, pos, Pp, gZp, gbp, nt in out:
        got_P[pos] = Pp
        got_gZ[start:stop] = gZp
        g_b += gbp
        n_targets.append(nt)
    assert np.array_equal(got_P, P)
    assert np.array_equal(got_gZ, g_Z)
    assert np.allclose(g_b, g_pre.astype(np.float64).sum(0), rtol=1e-5, atol=1e-4)
    assert sum(n_targets) == targets.size
    if world >= 4:
        assert n_targets[-1] == 0  # a rank with no targets


def _chunk_agree_worker(rank, world, port, K, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from graphconvgeo_amd.distributed import RowPartitionedCSR
        H, bounds = _unequal_graph()
        Z = np.random.default_rng(7).standard_normal((H.shape[0], K)).astype(np.float32)
        part = RowPartitionedCSR(H, rank, world, "cpu", local_spmm=_oracle_spmm,
                                 exchange="halo", bounds=bounds)
        c = part.choose_chunks(K)
        Zl = torch.from_numpy(part.local_rows(Z).copy())
        Y = torch.empty((part.n_local, K))
        part.spmm_pipelined(Zl, Y, n_chunks="auto")  # one all_to_all per chunk on every rank
        out = [None] * world
        dist.all_gather_object(out, (rank, c, part.halo_rows, part.start, part.stop, Y.numpy()))
        if rank == 0:
            q.put(out)
    finally:
        dist.destroy_process_group()


def _unequal_graph():
    """A 2000-node power-law graph plus 1000 isolated self-loop nodes, split into unequal
    blocks: the last rank's block references no remote row (its halo is empty)."""
    import scipy.sparse as sps
    H = sps.block_diag((synthetic_graph(2000, 12000), sps.identity(1000, dtype=np.float32)),
                       format="csr").astype(np.float32)
    return H, np.array([0, 500, 1400, 2000, 3000])


def test_auto_chunks_agree_across_ranks():
    """the auto column-chunk count must be the same on every rank, or ranks
    issue different numbers and widths of collectives. Unequal blocks, halo exchange, K = 136
    (2 chunks possible), and one rank with an empty halo -- whose own numbers alone would say
    'nothing to hide, 1 chunk' while the others want 2. Every rank picks the same count and
    the pipelined product equals the unpartitioned one."""
    from oracle import gcn_oracle as O
    from graphconvgeo_amd.distributed import PartitionPlan, pipeline_time
    K, world = 136, 4
    H, bounds = _unequal_graph()
    plan = PartitionPlan(H, world, bounds)
    assert plan.rows_in("halo")[-1] == 0
    # the rank-local model of round 4 would disagree here (the premise of the test)
    assert pipeline_time(0.0, 1.0, 1) < pipeline_time(0.0, 1.0, 2)
    (out,) = _run_world(_chunk_agree_worker, world, K)
    chunks = {c for _r, c, *_ in out}
    assert len(chunks) == 1 and chunks == {plan.choose_chunks("halo", K)} == {2}
    assert out[-1][2] == 0  # the last rank's halo is empty
    Z = np.random.default_rng(7).standard_normal((H.shape[0], K)).astype(np.float32)
    ref = O.spmm_f32(H, Z)
    got = np.zeros_like(ref)
    for _r, _c, _h, start, stop, Y in out:
        got[start:stop] = Y
    assert np.array_equal(got, ref)


def test_local_targets_keeps_order_and_duplicates():
    from graphconvgeo_amd.dist_train import local_targets
    pos, loc = local_targets(np.array([5, 1, 7, 5, 3, 9]), 3, 8)
    assert pos.tolist() == [0, 2, 3, 4] and loc.tolist() == [2, 4, 2, 0]


def _fit_loop_worker(rank, world, port, q):
    """RowPartitionedMLPCONV.fit's loop and the partition's probability gather over gloo, with a
    scripted CPU network in place of the HIP one (the numerics are tests/test_dist_train_gpu.py)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import scipy.sparse as sps
        from graphconvgeo_amd.dist_train import RowPartitionedGCN, RowPartitionedMLPCONV
        from graphconvgeo_amd.distributed import row_partition

        VAL = [5.0, 4.0, 3.0, 3.5, 3.2, 3.9, 4.0, 4.1, 4.2]  # dev loss at epochs 0, 5, 10, ...

        class _Part:
            def __init__(self, H, rank, world):
                self.n, self.world, self.device = H.shape[0], world, torch.device("cpu")
                self.bounds = row_partition(H.indptr, world)
                self.start, self.stop = int(self.bounds[rank]), int(self.bounds[rank + 1])

        class ScriptedNet(RowPartitionedGCN):
            def __init__(self, H, X, train_idx, Y, hidden, n_classes, rank, world, device,
                         group=None, **kw):
                self.rank, self.world, self.group = rank, world, group
                self.device = torch.device(device)
                self.part = _Part(H, rank, world)
                self.n_classes = n_classes
                self._y_all = np.asarray(Y)
                self.targets = {}
                self.add_targets("train", train_idx)
                self.W = torch.nn.Parameter(torch.zeros(2))
                self.b1 = torch.nn.Parameter(torch.zeros(1))
                self.b2 = torch.nn.Parameter(torch.zeros(1))
                self.params = [self.W, self.b1, self.W, self.b2]
                self.epoch = 0

            def make_optimizer(self, lr=4e-3):
                return None

            def train_step(self, opt):
                with torch.no_grad():
                    self.W += 1.0  # the parameters after epoch n hold n + 1
                self.epoch += 1
                # each rank's share: its targets / total -> the all-reduced mean is 1.0
                share = torch.tensor([len(self.targets["train"]) / self.targets["train"].total,
                                      0.5 * len(self.targets["train"]) / self.targets["train"].total])
                dist.all_reduce(share)
                return share[0], share[1]

            def evaluate(self, name, penalty=True):
                k = (self.epoch - 1) // 5
                v = torch.tensor([VAL[min(k, len(VAL) - 1)] / self.world, 0.1 * k / self.world])
                dist.all_reduce(v)
                if name == "_accuracy":  # accuracy(): fraction of hits of the given labels
                    tg = self.targets[name]
                    hits = (tg.y.to(torch.float64) == 1).to(torch.float64)
                    w = tg.weight.to(torch.float64) if tg.weight is not None else 1.0
                    a = torch.tensor([float((hits * w).sum()) / tg.total], dtype=torch.float64)
                    dist.all_reduce(a)
                    return v[0], a[0]
                return v[0], v[1]

            def local_probabilities(self, name):
                tg = self.targets[name]
                node = torch.as_tensor(tg.idx[tg.pos], dtype=torch.float32)
                out = torch.zeros((len(tg), self.n_classes))
                out[:, 0] = node
                out[:, 1] = float(self.rank)
                out[torch.arange(len(tg)), 2 + (tg.idx[tg.pos] % (self.n_classes - 2))] = 1e3
                return out

        H = synthetic_graph(600, 3000)
        X = sps.random(600, 20, density=0.1, format="csr", random_state=1, dtype=np.float32)
        Y = np.random.default_rng(2).integers(0, 6, size=600)
        train = np.random.default_rng(3).choice(400, 500).astype(np.int32)  # with replacement
        dev_i = np.arange(400, 500, dtype=np.int32)
        test_i = np.random.default_rng(4).permutation(600)[:70].astype(np.int32)
        clf = RowPartitionedMLPCONV(n_epochs=40, hidden_layer_size=4, report_k_epoch=5,
                                    early_stopping_max_down=3, device="cpu",
                                    network_factory=ScriptedNet)
        clf.fit(X, train, dev_i, test_i, Y, H)
        proba = clf.predict_proba("test")
        pred = clf.predict("test")
        acc = clf.accuracy("test", (Y[test_i] == 1).astype(np.int64))
        q.put((rank, clf.history, float(clf.params[0].detach()[0]), clf.best_dev_loss, proba, pred, acc))
    finally:
        dist.destroy_process_group()


def test_row_partitioned_fit_loop_and_gather():
    """RowPartitionedMLPCONV.fit over gloo world-2: validation every report_k_epoch from the
    all-reduced dev loss, best-parameter restore, early stopping after early_stopping_max_down
    non-improving validations (mlpconv.py:296-318 as graphconvgeo_amd.mlpconv.MLPCONV.fit does
    it), identical on both ranks; predict_proba gathers the test rows to rank 0 in the original
    target order; accuracy is the global hit fraction on every rank."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fit_loop_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted((q.get(timeout=120) for _ in range(world)), key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, hist0, w0, best0, proba0, pred0, acc0), (_, hist1, w1, best1, proba1, pred1, acc1) = out
    assert hist0 == hist1 and w0 == w1 and best0 == best1 and acc0 == acc1
    vals = [h["val_loss"] for h in hist0 if "val_loss" in h]
    # dev losses 5, 4, 3 (best, epoch 10), then 3.5, 3.2, 3.9 -> 3 non-improving, then 4.0 is
    # the 4th: n_down 4 > 3 stops at epoch 30
    assert [round(v, 6) for v in vals] == [5.0, 4.0, 3.0, 3.5, 3.2, 3.9, 4.0]
    assert hist0[-1]["epoch"] == 30 and len(hist0) == 31
    assert all(abs(h["train_loss"] - 1.0) < 1e-6 and abs(h["train_acc"] - 0.5) < 1e-6
               for h in hist0)
    assert w0 == 11.0  # parameters restored to the ones after epoch 10
    assert proba1 is None and pred1 is None
    test_i = np.random.default_rng(4).permutation(600)[:70]
    assert np.array_equal(proba0[:, 0], test_i.astype(np.float32))  # original target order
    assert set(np.unique(proba0[:, 1])) == {0.0, 1.0}  # rows from both ranks
    assert np.array_equal(pred0, 2 + test_i % 4)
    Y = np.random.default_rng(2).integers(0, 6, size=600)
    assert abs(acc0 - float((Y[test_i] == 1).mean())) < 1e-6


def test_mode_resolved_once_for_all_ranks():
    """'auto' at N > 1 is the mode the whole graph resolves to (RowPartitionedCSR.resolve_mode),
    the same on every rank and at every N, so a scaling series runs one arithmetic; what each
    row block alone would pick is reported in block_modes; explicit modes pass through."""
    from graphconvgeo_amd import sparse as gs
    from graphconvgeo_amd.distributed import RowPartitionedCSR
    H = synthetic_graph(60_000, 600_000)  # power-law: hub rows
    lens = np.diff(H.indptr)
    whole = gs.auto_mode(H.shape[0], H.nnz, int(lens.max()))
    for P in (2, 4):
        got = []
        for r in range(P):
            part = RowPartitionedCSR(H, r, P, "cpu", local_spmm=_oracle_spmm, exchange="allgather")
            got.append((part.resolve_mode("auto"), tuple(part.block_modes)))
            assert part.resolve_mode("fast") == "fast"
        assert len(set(got)) == 1  # every rank the same mode and the same per-block view
        mode, blocks = got[0]
        assert mode == whole and len(blocks) == P
        for q, m in enumerate(blocks):
            b = RowPartitionedCSR(H, q, P, "cpu", local_spmm=_oracle_spmm).bounds
            L = lens[b[q]:b[q + 1]]
            assert m == gs.auto_mode(L.size, int(L.sum()), int(L.max()))


def test_chunk_count_model():
    """RowPartitionedCSR.choose_chunks: 1 with nothing to hide (world 1); the pipeline model's
    optimum otherwise -- exchange-bound steps take the most chunks, chunks stay >= 64 columns --
    and pipeline_time itself: 1 chunk = exchange + SpMM, more chunks hide the shorter phase."""
    from graphconvgeo_amd.distributed import (MAX_CHUNKS, RowPartitionedCSR, pipeline_time)
    assert pipeline_time(2.0, 1.0, 1) == 3.0
    assert pipeline_time(2.0, 1.0, 4) < pipeline_time(2.0, 1.0, 2) < 3.0
    assert pipeline_time(0.0, 1.0, 4) > pipeline_time(0.0, 1.0, 1)  # nothing to hide: chunks cost
    H = synthetic_graph(20_000, 160_000)
    one = RowPartitionedCSR(H, 0, 1, "cpu", local_spmm=_oracle_spmm)
    assert one.choose_chunks(300) == 1
    p = RowPartitionedCSR(H, 0, 4, "cpu", local_spmm=_oracle_spmm, exchange="allgather")
    assert p.choose_chunks(300) == MAX_CHUNKS   # the exchange dwarfs a 20k-node local SpMM
    assert p.choose_chunks(100) == 1            # one 64-column chunk at most
    assert p.choose_chunks(130) == 2
    p.chunks_override = 3
    assert p._n_chunks("auto", 300) == 3 and p._n_chunks(2, 300) == 2


def test_row_partition_hub_weight():
    """The cost model: hub rows (longer than hub_nnz) weighted by hub_weight move the cuts away
    from the blocks that hold them; weight 1 is the round-3 nnz + 2 * rows balance."""
    from graphconvgeo_amd.distributed import row_partition
    lens = np.array([1] * 1000 + [5000] + [1] * 9000)
    indptr = np.concatenate([[0], np.cumsum(lens)])
    b1 = row_partition(indptr, 2)
    cost = indptr + 2 * np.arange(indptr.size)
    assert abs(cost[b1[1]] - cost[-1] / 2) <= 5000 + 3
    b3 = row_partition(indptr, 2, hub_weight=3.0)
    assert b3[1] <= b1[1]  # the block holding the hub row gets fewer rows
    assert row_partition(indptr, 2, hub_weight=1.0).tolist() == b1.tolist()


def test_target_rows_backward_operator_structure():
    """TargetRowsBackward on one rank of a 3-way partition: the operator is H_q with every column
    outside the global distinct targets dropped, columns remapped to each owner's block of the
    exchange layout; every rank's distinct targets come from the global list (no communication);
    the operator times the scattered-then-gathered gradient equals H_q times the full scatter."""
    from oracle import gcn_oracle as O
    from graphconvgeo_amd.distributed import RowPartitionedCSR, TargetRows
    n, e = 3000, 20000
    H = synthetic_graph(n, e)
    rng = np.random.default_rng(9)
    targets = rng.integers(0, 2000, size=1800).astype(np.int32)  # bunched on the first ranks
    g_full = np.zeros((n, 8), np.float32)
    G = rng.standard_normal((targets.size, 8)).astype(np.float32)
    O.scatter_add_f32(g_full, targets, G)
    for r in range(3):
        part = RowPartitionedCSR(H, r, 3, "cpu", local_spmm=_oracle_spmm, exchange="allgather")
        tg = TargetRows(targets, part)
        op = part.target_backward(tg)
        assert part.target_backward(tg) is op
        counts = op.layout.counts
        assert counts == [np.unique(targets[(targets >= part.bounds[q]) &
                                            (targets < part.bounds[q + 1])]).size for q in range(3)]
        # operand: each rank's distinct rows of the scattered gradient, in its block
        operand = np.zeros((3 * op.layout.pad, 8), np.float32)
        for q, d in enumerate(tg.block_distinct):
            operand[q * op.layout.pad:q * op.layout.pad + d.size] = g_full[d]
        got = O.spmm_f32(op.host, operand)
        want = O.spmm_f32(H[part.start:part.stop], g_full)
        assert np.array_equal(got, want)
        assert op.nnz < part.nnz_local
    # bunched targets: the exact-count mesh is chosen over the padded all-gather
    assert op.layout.method == "mesh"


def test_host_symmetry_check():
    """distributed.host_is_symmetric: the symmetric D^-1/2 (A+I) D^-1/2 (canonical, and with
    every row's storage order shuffled) is symmetric; the reference's row-normalized
    D^-1 (A+I) (main.py:451-456) is not; a rectangular matrix never is."""
    import scipy.sparse as sps
    from graphconvgeo_amd.distributed import host_is_symmetric
    H = synthetic_graph(2000, 12000)
    assert host_is_symmetric(H)
    Hs = H.copy()
    rng = np.random.default_rng(0)
    for i in range(Hs.shape[0]):
        a, b = Hs.indptr[i], Hs.indptr[i + 1]
        p = rng.permutation(b - a) + a
        Hs.indices[a:b], Hs.data[a:b] = Hs.indices[p].copy(), Hs.data[p].copy()
    assert host_is_symmetric(Hs)
    assert not host_is_symmetric(_operator(2000, 12000, True))
    assert not host_is_symmetric(sps.random(20, 30, 0.2, format="csr", dtype=np.float32))


def test_plan_of_another_graph_is_refused():
    """RowPartitionedCSR(H, plan=...) used plan.H silently; a plan built from
    another graph is now an error (the same graph, as another object, is accepted)."""
    from graphconvgeo_amd.distributed import PartitionPlan, RowPartitionedCSR
    H1, H2 = synthetic_graph(1500, 8000), synthetic_graph(1500, 8000, seed=5)
    plan = PartitionPlan(H1, 2)
    with pytest.raises(ValueError):
        RowPartitionedCSR(H2, 0, 2, "cpu", local_spmm=_oracle_spmm, plan=plan)
    part = RowPartitionedCSR(H1.copy(), 0, 2, "cpu", local_spmm=_oracle_spmm, plan=plan)
    assert part.plan is plan
    assert RowPartitionedCSR(None, 1, 2, "cpu", local_spmm=_oracle_spmm, plan=plan).start == plan.bounds[1]


def test_target_backward_operator_freed_with_its_list():
    """the backward operator is cached on the target list and holds no reference
    back to it, so dropping the list frees both by reference counting (no cycle for the GC)."""
    import gc
    import weakref
    from graphconvgeo_amd.distributed import RowPartitionedCSR, TargetRows
    H = synthetic_graph(1500, 8000)
    part = RowPartitionedCSR(H, 0, 2, "cpu", local_spmm=_oracle_spmm, exchange="allgather")
    tg = TargetRows(np.arange(0, 600, 3, dtype=np.int32), part)
    op = part.target_backward(tg)
    assert tg._backward_op is op and not hasattr(op, "targets")
    ref_op, ref_tg = weakref.ref(op), weakref.ref(tg)
    gc.disable()
    try:
        del op, tg
        assert ref_tg() is None and ref_op() is None
    finally:
        gc.enable()
