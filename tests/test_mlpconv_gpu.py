"""GPU trainer (MLPCONV, mlpconv.py:121-352) against the float64 oracle trajectory."""
import numpy as np
import pytest

from graphconvgeo_amd.mlpconv import MLPCONV
from graphconvgeo_amd.synth import glorot_uniform, synthetic_features, synthetic_graph
from oracle import gcn_oracle as O

pytestmark = pytest.mark.gpu


def problem(n=4000, e=30000, f=300, k=48, c=9, seed=0):
    H = synthetic_graph(n, e)
    X = synthetic_features(n, f, nnz_per_row=20, empty_frac=0.02)
    rng = np.random.default_rng(seed)
    Y = rng.integers(0, c, size=n)
    # labels correlated with features so training makes progress
    Y = (np.asarray(X[:, :c].argmax(axis=1)).ravel() + (rng.random(n) < 0.2)) % c
    n_tr, n_dev = int(0.6 * n), int(0.2 * n)
    train = np.random.default_rng(77).choice(n_tr, size=n_tr).astype(np.int32)  # with replacement
    dev = np.arange(n_tr, n_tr + n_dev, dtype=np.int32)
    test = np.arange(n_tr + n_dev, n, dtype=np.int32)
    W1, W2 = glorot_uniform(f, k), glorot_uniform(k, c, seed=3)
    b1, b2 = np.zeros(k, np.float32), np.zeros(c, np.float32)
    return H, X, Y, train, dev, test, (W1, b1, W2, b2)


def test_mlpconv_trajectory_matches_oracle(cuda):
    H, X, Y, train, dev, test, init = problem()
    coefs = (1e-5, 1e-5)
    clf = MLPCONV(n_epochs=15, hidden_layer_size=48, regul_coefs=coefs, init_parameters=init,
                  device=cuda, report_k_epoch=5)
    clf.fit(X, train, dev, test, Y, H)
    hist, params = O.mlpconv_train(X, H, Y, train, dev, *init, n_epochs=15, regul_coefs=coefs,
                                   report_k_epoch=5)
    got = np.array([h["train_loss"] for h in clf.history])
    ref = np.array([h["train_loss"] for h in hist])
    assert got.shape == ref.shape
    assert np.abs(got - ref).max() < 1e-4 * max(1.0, np.abs(ref).max()), (got, ref)
    assert ref[-1] < ref[0]  # it trains
    gv = [h["val_loss"] for h in clf.history if "val_loss" in h]
    rv = [h["val_loss"] for h in hist if "val_loss" in h]
    assert np.allclose(gv, rv, rtol=1e-4, atol=1e-5)


def test_mlpconv_api(cuda, tmp_path):
    H, X, Y, train, dev, test, init = problem(n=2000, e=12000, f=150, k=16, c=5)
    clf = MLPCONV(n_epochs=21, hidden_layer_size=16, device=cuda, seed=1,
                  early_stopping_max_down=5, model_file=str(tmp_path / "best.pt"))
    clf.fit(X, train, dev, test, Y, H)
    pred = clf.predict("test")
    proba = clf.predict_proba("test")
    assert pred.shape == (len(test),) and proba.shape == (len(test), int(Y.max()) + 1)
    assert np.allclose(proba.sum(axis=1), 1.0, atol=1e-5)
    assert np.array_equal(pred, proba.argmax(axis=1))
    acc = clf.accuracy("test", Y[test])
    assert abs(acc - float((pred == Y[test]).mean())) < 1e-6
    assert clf.score(X, "test", Y[test]) == acc  # mlpconv.py:348 signature
    assert 0.0 <= clf.best_dev_acc <= 1.0  # final dev evaluation, mlpconv.py:316-318
    assert (tmp_path / "best.pt").exists()
    with pytest.raises(ValueError):
        clf.predict("nope")


def test_mlpconv_propagate_first_order(cuda):
    """Reassociated layer 2 ((H.h)[idx].W2) tracks the reference-order oracle within tolerance."""
    H, X, Y, train, dev, test, init = problem(c=60)  # C > K: auto picks propagate_first
    coefs = (1e-5, 1e-5)
    clf = MLPCONV(n_epochs=12, hidden_layer_size=48, regul_coefs=coefs, init_parameters=init,
                  device=cuda, report_k_epoch=4, order="auto")
    clf.fit(X, train, dev, test, Y, H)
    assert clf.l_out.order == "propagate_first"
    hist, _ = O.mlpconv_train(X, H, Y, train, dev, *init, n_epochs=12, regul_coefs=coefs,
                              report_k_epoch=4)
    got = np.array([h["train_loss"] for h in clf.history])
    ref = np.array([h["train_loss"] for h in hist])
    assert np.abs(got - ref).max() < 1e-4 * max(1.0, np.abs(ref).max()), (got, ref)


@pytest.mark.parametrize("order", ["reference", "propagate_first"])
def test_mlpconv_hip_graph_equals_eager(cuda, order):
    """A captured epoch replays the eager one bit for bit; in the propagate-first order the
    capture holds the fused MFMA output kernel and the padded-weight copy it reads (re-copied on
    every replay, since Adam moves W2 between replays)."""
    H, X, Y, train, dev, test, init = problem(n=3000, e=20000, f=200, k=32, c=7)
    kw = dict(n_epochs=11, hidden_layer_size=32, regul_coefs=(1e-5, 1e-5), init_parameters=init,
              device=cuda, report_k_epoch=5, order=order)
    a = MLPCONV(**kw).fit(X, train, dev, test, Y, H)
    b = MLPCONV(use_graph=True, **kw).fit(X, train, dev, test, Y, H)
    assert [h["train_loss"] for h in a.history] == [h["train_loss"] for h in b.history]
    # validation runs eagerly between replays: it must see the weights of the latest replay
    # (a padded-weight copy cached during capture would be one Adam step behind)
    assert [h.get("val_loss") for h in a.history] == [h.get("val_loss") for h in b.history]
    assert a.best_dev_acc == b.best_dev_acc
    for pa, pb in zip(a.get_params(), b.get_params()):
        assert np.array_equal(pa, pb)  # replayed graph == eager, bit for bit


def test_main_mlpconv_call_pattern(cuda):
    """The exact constructor / fit / accuracy / predict calls of tensormain.main_mlpconv
    (tensormain.py:232-244), with the import swapped for graphconvgeo_amd's MLPCONV."""
    H, X, Y, train, dev, test, _init = problem(n=2500, e=15000, f=200, k=24, c=6)
    regul, hidden_size, batch_size, dropout_coefs, dtype = 1e-6, 24, 500, [0.5, 0.5], "float32"
    clf = MLPCONV(n_epochs=30, batch_size=batch_size, init_parameters=None, complete_prob=False,
                  add_hidden=True, regul_coefs=[regul, regul], save_results=False,
                  hidden_layer_size=hidden_size, drop_out=False, dropout_coefs=dropout_coefs,
                  early_stopping_max_down=5, loss_name='log', nonlinearity='rectify', dtype=dtype)
    clf.fit(X, train, dev, test, Y, H)
    acc = clf.accuracy(dataset_partition='test', y_true=Y[test].astype('int32'))
    y_pred = clf.predict(dataset_partition='test')
    assert 0.0 <= acc <= 1.0 and y_pred.shape == (len(test),)
    assert acc > 1.5 / 6  # learns beyond chance on feature-correlated labels


def test_default_init_is_lasagne_glorot_from_numpy_global_stream(cuda):
    """init_parameters=None: W1 then W2 from np.random after np.random.seed(77), as
    main_mlpconv seeds it (tensormain.py:227) before MLPCONV's DenseLayers draw them
    (mlpconv.py:205-217). Parity unpinned: Lasagne is not importable here."""
    H, X, Y, train, dev, test, _ = problem(n=1500, e=9000, f=120, k=16, c=5)
    np.random.seed(77)
    clf = MLPCONV(n_epochs=0, hidden_layer_size=16, device=cuda)
    clf.fit(X, train, dev, test, Y, H)
    rs = np.random.RandomState(77)
    a1 = np.sqrt(3) * np.sqrt(2.0 / (120 + 16))
    a2 = np.sqrt(3) * np.sqrt(2.0 / (16 + 5))
    W1 = rs.uniform(-a1, a1, size=(120, 16)).astype(np.float32)
    W2 = rs.uniform(-a2, a2, size=(16, 5)).astype(np.float32)
    got = clf.get_params()
    assert np.array_equal(got[0], W1) and np.array_equal(got[2], W2)
    assert not got[1].any() and not got[3].any()  # b = Constant(0.)


def test_fused_adam_matches_elementwise_formula(cuda):
    """gcg_adam_step_f32 (one launch per parameter) against lasagne.updates.adam written out
    elementwise in float64, over several steps (mlpconv.py:263)."""
    import torch
    from graphconvgeo_amd.mlpconv import LasagneAdam
    g0 = torch.Generator(device=cuda).manual_seed(3)
    ps = [torch.nn.Parameter(torch.randn(s, generator=g0, device=cuda)) for s in ((300, 7), (7,), (5000,))]
    ref = [p.detach().double().clone() for p in ps]
    m = [torch.zeros_like(r) for r in ref]
    v = [torch.zeros_like(r) for r in ref]
    opt = LasagneAdam(ps)
    for t in range(1, 6):
        grads = [torch.randn(p.shape, generator=g0, device=cuda) for p in ps]
        for p, g in zip(ps, grads):
            p.grad = g.clone()
        opt.step()
        a = 4e-3 * np.sqrt(1 - 0.999 ** t) / (1 - 0.9 ** t)
        for i, g in enumerate(grads):
            g = g.double()
            m[i] = 0.9 * m[i] + 0.1 * g
            v[i] = 0.999 * v[i] + 0.001 * g * g
            ref[i] = ref[i] - a * m[i] / (v[i].sqrt() + 1e-8)
        for p, r in zip(ps, ref):
            assert float((p.detach().double() - r).abs().max()) < 1e-6, t
    # an in-place update as far as torch knows: version counters move (weight-copy caches)
    assert all(p._version >= 5 for p in ps)


@pytest.mark.parametrize("order", ["reference", "propagate_first"])
def test_distinct_targets_equal_full_target_list(cuda, order):
    """Targets drawn with replacement (tensormain.py:226): the output layer on the distinct
    rows with multiplicity weights gives the loss, accuracy and gradients of the full list
    (within fp32 rounding: a multiplicity times one copy vs the copies added in order)."""
    import torch

    H, X, Y, train, dev, test, init = problem()
    assert np.unique(train).size < train.size
    res = {}
    for distinct in (False, True):
        clf = MLPCONV(n_epochs=0, hidden_layer_size=48, regul_coefs=(1e-5, 1e-5),
                      init_parameters=init, device=cuda, mode="ordered", order=order)
        clf.fit(X, train, dev, test, Y, H)
        clf.distinct_targets = distinct
        y = torch.as_tensor(Y[train].astype(np.int32), device=cuda)
        loss, acc = clf._loss_acc(clf.rows["train"], y)
        loss.backward()
        res[distinct] = (float(loss), float(acc), [p.grad.cpu().numpy() for p in clf.params])
    (l0, a0, g0), (l1, a1, g1) = res[False], res[True]
    assert abs(l1 - l0) <= 1e-6 * abs(l0)
    assert abs(a1 - a0) <= 1e-6
    for x, z in zip(g0, g1):
        assert np.abs(x - z).max() <= 1e-5 * max(1.0, np.abs(x).max())


@pytest.mark.parametrize("pattern", ["one_row", "no_repeats", "heavy"])
def test_distinct_targets_edge_cases(cuda, pattern):
    """Distinct-target weighting at the edges: every target the same row (one distinct row of
    multiplicity T), no repeats (the plain path), and a few rows drawn very often."""
    import torch

    H, X, Y, train, dev, test, init = problem(n=1500, e=9000)
    n_tr = 900
    if pattern == "one_row":
        tgt = np.full(400, 17, dtype=np.int32)
    elif pattern == "no_repeats":
        tgt = np.random.default_rng(3).permutation(n_tr)[:500].astype(np.int32)
    else:
        tgt = np.random.default_rng(4).choice(np.arange(5), size=700).astype(np.int32)
    res = {}
    for distinct in (False, True):
        clf = MLPCONV(n_epochs=0, hidden_layer_size=48, regul_coefs=(1e-5, 1e-5),
                      init_parameters=init, device=cuda, mode="ordered", order="propagate_first")
        clf.fit(X, tgt, dev, test, Y, H)
        clf.distinct_targets = distinct
        y = torch.as_tensor(Y[tgt].astype(np.int32), device=cuda)
        loss, acc = clf._loss_acc(clf.rows["train"], y)
        loss.backward()
        res[distinct] = (float(loss), float(acc), [p.grad.cpu().numpy() for p in clf.params])
    assert (clf.rows["train"].distinct() is None) == (pattern == "no_repeats")
    (l0, a0, g0), (l1, a1, g1) = res[False], res[True]
    assert abs(l1 - l0) <= 1e-6 * abs(l0) and abs(a1 - a0) <= 1e-6
    for x, z in zip(g0, g1):
        assert np.abs(x - z).max() <= 1e-5 * max(1.0, np.abs(x).max())


@pytest.mark.parametrize("order", ["reference", "propagate_first"])
@pytest.mark.parametrize("use_graph", [False, True])
def test_training_raises_no_stream_warnings(cuda, order, use_graph):
    """The side-stream weight gradients leave no cross-stream accumulation behind: every
    gradient reaching W2 (its product gradient and its penalty gradient) is produced on the
    stream its AccumulateGrad node lives on, so torch's stream-mismatch warning never fires
    (eager epochs and a captured HIP graph alike)."""
    import warnings

    H, X, Y, train, dev, test, init = problem(n=2000, e=12000, f=150, k=16, c=5)
    with warnings.catch_warnings(record=True) as caught:
        warnings.simplefilter("always")
        MLPCONV(n_epochs=11, hidden_layer_size=16, regul_coefs=(1e-5, 1e-5), init_parameters=init,
                device=cuda, report_k_epoch=5, order=order, use_graph=use_graph
                ).fit(X, train, dev, test, Y, H)
    msgs = [str(w.message) for w in caught if "stream" in str(w.message).lower()]
    assert not msgs, msgs[:2]
