"""BASELINE config 3 at full size: one 2-layer GCN forward + backward (an MLPCONV epoch's
f_train, mlpconv.py:293-295, as tensormain.py:232-237 runs it) on the Twitter-US-scale
synthetic problem -- N = 450k users, E = 5M edges, F = 10k features, K = 300, C = 256 --
in both layer-2 orders, against the oracle:

  h        sampled rows (random, hubs, shortest) bitwise vs the float32 oracle chain
           rectify(H . (X . W1) + b1) (scipy csr_matvecs order; mode='ordered')
  P        sampled rows within 1e-5 of the float64 forward (the dense projection is an
           f32 MFMA/BLAS product: within rounding, not bitwise)
  loss     within 1e-5 (relative) of the float64 loss (CE mean + L1/L2 shares)
  dW1 dW2 db1 db2  the full gradients against the float64 Theano-rule backward
           (gcn_oracle.gcn_backward): max |err| <= 1e-5 * max(1, max |ref|) and
           ||err||_F <= 1e-4 ||ref||_F (fp32 sums of up to ~10^5 terms).
The float64 oracle runs once for the module (~1 min of host time)."""
import numpy as np
import pytest
import torch

from graphconvgeo_amd.mlpconv import MLPCONV
from graphconvgeo_amd.synth import CONFIGS, glorot_uniform, synthetic_features, synthetic_graph
from oracle import gcn_oracle as O

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(900)]
COEFS = (5e-5, 5e-5)  # MLPCONV's default regul_coefs (mlpconv.py:128)


@pytest.fixture(scope="module")
def us():
    cfg = CONFIGS["twitter-us"]
    n, F, K, C = cfg.n_nodes, cfg.n_features, cfg.hidden, cfg.n_classes
    H = synthetic_graph(n, cfg.n_edges)
    X = synthetic_features(n, F, nnz_per_row=64, empty_frac=0.01)
    rng = np.random.default_rng(77)
    Y = rng.integers(0, C, size=n)
    n_tr = int(0.6 * n)
    train = rng.choice(n_tr, size=n_tr).astype(np.int32)  # with replacement, tensormain.py:226
    dev = np.arange(n_tr, int(0.8 * n), dtype=np.int32)
    test = np.arange(int(0.8 * n), n, dtype=np.int32)
    W1, W2 = glorot_uniform(F, K), glorot_uniform(K, C, seed=9)
    b1 = np.random.default_rng(3).standard_normal(K).astype(np.float32) * 0.01
    b2 = np.zeros(C, np.float32)
    lens = np.diff(H.indptr)
    sample = np.unique(np.concatenate([np.random.default_rng(4).integers(0, n, 3000),
                                       np.argsort(lens)[-40:], np.argsort(lens)[:40]]))
    # float32 oracle chain for the bitwise h rows
    Z1_32 = O.spmm_f32(X, W1)
    h_rows = O.spmm_f32(H, Z1_32, bias=b1, act="relu", rows=sample)
    del Z1_32
    f64 = O.gcn_forward(X, H, W1, b1, W2, b2, train)
    loss64 = O.gcn_loss(f64["P"], Y[train], W1, W2, COEFS)
    g64 = O.gcn_backward(X, H, W1, W2, f64, train, Y[train], regul_coefs=COEFS)
    pos = np.random.default_rng(5).integers(0, train.size, 3000)
    return dict(cfg=cfg, H=H, X=X, Y=Y, train=train, dev=dev, test=test,
                init=(W1, b1, W2, b2), sample=sample, h_rows=h_rows, pos=pos,
                P64=f64["P"][pos], loss64=float(loss64),
                g64={k: g64[k] for k in ("W1", "b1", "W2", "b2")})


@pytest.mark.parametrize("order", ["reference", "propagate_first"])
def test_twitter_us_fwd_bwd(cuda, us, order):
    cfg = us["cfg"]
    clf = MLPCONV(n_epochs=0, hidden_layer_size=cfg.hidden, regul_coefs=COEFS,
                  init_parameters=us["init"], device=cuda, mode="ordered", order=order)
    clf.fit(us["X"], us["train"], us["dev"], us["test"], us["Y"], us["H"])
    rows = clf.rows["train"]
    with torch.no_grad():
        h = clf.l_hid1(clf.Xd)
        got_h = h[torch.as_tensor(us["sample"], device=cuda)].cpu().numpy()
        P = clf._probabilities(rows)[torch.as_tensor(us["pos"], device=cuda)].cpu().numpy()
    assert np.array_equal(got_h, us["h_rows"])  # bitwise scipy float32 chain
    assert np.abs(P - us["P64"]).max() < 1e-5
    y = torch.as_tensor(us["Y"][us["train"]].astype(np.int32), device=cuda)
    loss, _acc = clf._loss_acc(rows, y)
    loss.backward()
    assert abs(float(loss.detach()) - us["loss64"]) <= 1e-5 * max(1.0, abs(us["loss64"]))
    for p, k in zip(clf.params, ("W1", "b1", "W2", "b2")):
        got = p.grad.detach().cpu().numpy().astype(np.float64)
        ref = us["g64"][k]
        err = got - ref
        assert np.abs(err).max() <= 1e-5 * max(1.0, np.abs(ref).max()), (k, np.abs(err).max())
        assert np.linalg.norm(err) <= 1e-4 * np.linalg.norm(ref), (k, np.linalg.norm(err) / np.linalg.norm(ref))
