"""A non-symmetric graph operator through the trainer.

The reference's MLPCONV.fit(X, ..., Y, H) takes any H (mlpconv.py:152,173,205-217), and Theano
back-propagates S.dot(H, Z) as H^T . gz whatever H is. The reference itself builds one
non-symmetric operator: the row-l1-normalized D^-1 (A+I) of main.py:451-456
(oracle.gcn_oracle.row_normalize_l1). Here: DeviceCSR.check_symmetric decides once on the
device; MLPCONV, GCN and the row-partitioned trainer back-propagate through H^T, against the
float64 Theano-rule gradients of gcn_oracle.gcn_backward (which uses H.T)."""
import os
import socket

import numpy as np
import pytest
import scipy.sparse as sps
import torch
import torch.multiprocessing as mp

from graphconvgeo_amd import sparse as gs
from graphconvgeo_amd.synth import synthetic_graph
from oracle import gcn_oracle as O
from test_mlpconv_gpu import problem

pytestmark = pytest.mark.gpu

COEFS = (1e-5, 1e-5)


def rownorm_problem(**kw):
    H, X, Y, train, dev, test, init = problem(**kw)
    A = H.copy()
    A.data[:] = 1.0
    Hr = O.row_normalize_l1(A)
    assert (abs(Hr - Hr.T) > 0).nnz > 0  # genuinely non-symmetric
    return Hr, X, Y, train, dev, test, init


def _grad_bar(got, ref):
    return np.abs(got - ref).max() <= 1e-5 * max(1.0, np.abs(ref).max())


def test_check_symmetric_decides_on_device(cuda):
    H = synthetic_graph(3000, 20000)
    A = gs.DeviceCSR.from_scipy(H, cuda)
    assert A.symmetric is None and A.transpose() is A and A.symmetric is True
    assert A._transpose is None  # the built transpose is dropped
    # the same symmetric matrix with every row's storage order shuffled: arrays differ, the
    # entry multisets do not
    rng = np.random.default_rng(0)
    Hs = H.copy()
    for i in range(Hs.shape[0]):
        a, b = Hs.indptr[i], Hs.indptr[i + 1]
        p = rng.permutation(b - a) + a
        Hs.indices[a:b], Hs.data[a:b] = Hs.indices[p].copy(), Hs.data[p].copy()
    Bs = gs.DeviceCSR.from_scipy(Hs, cuda)
    assert Bs.check_symmetric() and Bs.transpose() is Bs
    # D^-1 (A+I): not symmetric; the transpose is the stable CSR of H^T (scipy's .T.tocsr())
    Hr = O.row_normalize_l1(H)
    R = gs.DeviceCSR.from_scipy(Hr, cuda)
    T = R.transpose()
    assert R.symmetric is False and T is not R
    ref = Hr.T.tocsr()
    assert np.array_equal(T.indptr.cpu().numpy(), ref.indptr)
    assert np.array_equal(T.indices.cpu().numpy(), ref.indices)
    assert np.array_equal(T.data.cpu().numpy(), ref.data)
    # one value off the mirror breaks symmetry
    Hb = H.copy()
    Hb.data[5] *= 1.5
    assert not gs.DeviceCSR.from_scipy(Hb, cuda).check_symmetric()
    # declared by the caller: no check
    D = gs.DeviceCSR.from_scipy(Hr, cuda, symmetric=False)
    assert D.transpose() is not D
    # rectangular: never symmetric
    assert not gs.DeviceCSR.from_scipy(sps.random(20, 30, 0.2, format="csr", dtype=np.float32),
                                       cuda).check_symmetric()


@pytest.mark.parametrize("order", ["reference", "propagate_first"])
def test_mlpconv_gradients_rownorm_operator(cuda, order):
    """First-step gradients of MLPCONV on D^-1 (A+I) within 1e-5 * max(1, |ref|) of the
    float64 Theano-rule gradients (gcn_backward uses H^T)."""
    from graphconvgeo_amd.mlpconv import MLPCONV
    H, X, Y, train, dev, test, init = rownorm_problem(c=60)
    clf = MLPCONV(n_epochs=0, hidden_layer_size=48, regul_coefs=COEFS, init_parameters=init,
                  device=cuda, order=order)
    clf.fit(X, train, dev, test, Y, H)
    y = torch.as_tensor(Y[train].astype(np.int32), device=cuda)
    loss, _acc = clf._loss_acc(clf.rows["train"], y)
    loss.backward()
    assert clf.l_hid1.H.symmetric is False
    W1, b1, W2, b2 = init
    f = O.gcn_forward(X, H, W1, b1, W2, b2, train)
    g64 = O.gcn_backward(X, H, W1, W2, f, train, Y[train], regul_coefs=COEFS)
    assert abs(float(loss) - O.gcn_loss(f["P"], Y[train], W1, W2, COEFS)) < 1e-5
    for p, k in zip(clf.params, ("W1", "b1", "W2", "b2")):
        got = p.grad.cpu().numpy()
        assert _grad_bar(got, g64[k]), (k, np.abs(got - g64[k]).max())
    # the symmetric-H gradients would be measurably different here (the check matters)
    Hsym = sps.csr_matrix(H.T)
    gwrong = O.gcn_backward(X, Hsym, W1, W2, f, train, Y[train], regul_coefs=COEFS)
    assert not _grad_bar(gwrong["W1"], g64["W1"])


def test_mlpconv_trajectory_rownorm_operator(cuda):
    from graphconvgeo_amd.mlpconv import MLPCONV
    H, X, Y, train, dev, test, init = rownorm_problem()
    clf = MLPCONV(n_epochs=12, hidden_layer_size=48, regul_coefs=COEFS, init_parameters=init,
                  device=cuda, report_k_epoch=4)
    clf.fit(X, train, dev, test, Y, H)
    hist, _ = O.mlpconv_train(X, H, Y, train, dev, *init, n_epochs=12, regul_coefs=COEFS,
                              report_k_epoch=4)
    got = np.array([h["train_loss"] for h in clf.history])
    ref = np.array([h["train_loss"] for h in hist])
    assert np.abs(got - ref).max() < 1e-4 * max(1.0, np.abs(ref).max()), (got, ref)


def test_gcn_module_rownorm_operator(cuda):
    """layers.GCN (the 2-layer model) on D^-1 (A+I): CE gradients against gcn_backward."""
    from graphconvgeo_amd.layers import GCN
    H, X, Y, train, dev, test, (W1, b1, W2, b2) = rownorm_problem(c=60)
    net = GCN(H, X, X.shape[1], 48, 60, device=cuda, W1=W1, W2=W2)
    P = net(train)
    y = torch.as_tensor(Y[train].astype(np.int64), device=cuda)
    loss = -torch.log(P[torch.arange(len(train), device=cuda), y]).mean()
    loss.backward()
    f = O.gcn_forward(X, H, W1, b1, W2, b2, train)
    g64 = O.gcn_backward(X, H, W1, W2, f, train, Y[train], regul_coefs=(0.0, 0.0))
    for p, k in ((net.l_hid1.W, "W1"), (net.l_hid1.b, "b1"), (net.l_out.W, "W2"),
                 (net.l_out.b, "b2")):
        got = p.grad.cpu().numpy()
        assert _grad_bar(got, g64[k]), (k, np.abs(got - g64[k]).max())


def test_symmetric_operator_unchanged(cuda):
    """The symmetric D^-1/2 (A+I) D^-1/2 still back-propagates through H itself: no transpose
    is kept, and the gradients are bitwise those of an operator declared symmetric."""
    from graphconvgeo_amd.mlpconv import MLPCONV
    H, X, Y, train, dev, test, init = problem(n=2000, e=12000, f=150, k=16, c=5)
    grads = []
    for declared in (None, True):
        Hd = gs.DeviceCSR.from_scipy(H, cuda, symmetric=declared)
        clf = MLPCONV(n_epochs=0, hidden_layer_size=16, regul_coefs=COEFS, init_parameters=init,
                      device=cuda)
        clf.fit(X, train, dev, test, Y, Hd)
        y = torch.as_tensor(Y[train].astype(np.int32), device=cuda)
        loss, _ = clf._loss_acc(clf.rows["train"], y)
        loss.backward()
        assert Hd.symmetric is True and Hd._transpose is None
        grads.append([p.grad.cpu().numpy() for p in clf.params])
    for a, b in zip(*grads):
        assert np.array_equal(a, b)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _dist_worker(rank, world, port, order, exchange, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from graphconvgeo_amd.dist_train import RowPartitionedGCN
        H, X, Y, train, dev, test, (W1, b1, W2, b2) = rownorm_problem(c=60)
        model = RowPartitionedGCN(H, X, train, Y, hidden=48, n_classes=60, rank=rank,
                                  world=world, device="cuda:0", W1=W1, W2=W2, order=order,
                                  exchange=exchange, regul_coefs=COEFS)
        opt = model.make_optimizer()
        loss, _acc = model.train_step(opt)
        grads = [p.grad.detach().cpu().numpy().copy() for p in model.params]
        torch.cuda.synchronize()
        q.put((rank, model.symmetric, float(loss), grads))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("order,exchange", [("propagate_first", "halo"),
                                            ("reference", "allgather")])
def test_row_partitioned_rownorm_operator(cuda, order, exchange):
    """RowPartitionedGCN (2 ranks over gloo on one MI355X) on D^-1 (A+I): the backward runs
    through a partition of CSR(H^T) over the same row bounds; the all-reduced first-step
    gradients against gcn_backward."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dist_worker, args=(r, world, port, order, exchange, q))
             for r in range(world)]
    for p in procs:
        p.start()
    out = sorted((q.get(timeout=240) for _ in range(world)), key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    H, X, Y, train, dev, test, (W1, b1, W2, b2) = rownorm_problem(c=60)
    f = O.gcn_forward(X, H, W1, b1, W2, b2, train)
    g64 = O.gcn_backward(X, H, W1, W2, f, train, Y[train], regul_coefs=COEFS)
    for _r, sym, loss, grads in out:
        assert sym is False
        assert abs(loss - O.gcn_loss(f["P"], Y[train], W1, W2, COEFS)) < 1e-5
        for got, k in zip(grads, ("W1", "b1", "W2", "b2")):
            assert _grad_bar(got, g64[k]), (k, np.abs(got - g64[k]).max())
