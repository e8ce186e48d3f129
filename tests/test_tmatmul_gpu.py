"""GPU parity of DeviceCSR.tmatmul = A^T . G, the gradient of S.dot(X, W1) w.r.t. W1
(mlpconv.py:71; Theano's Dot grad x^T . gz). Columns of X denser than HYBRID_MIN_DENSITY go
through the split-K MFMA GEMM, the rest through the CSR(X^T) gather.

Bar: 'ordered' is bitwise the CSR(X^T) gather; the split ('fast', and 'auto' when the
transpose would split rows anyway) is within fp32 summation error of the float64 product:
|y - y64| <= 1e-5 * (|X|^T |G|) elementwise (parity unpinned beyond that: Theano's CPU
grad runs the same sum in scipy order)."""
import numpy as np
import pytest
import scipy.sparse as sps
import torch

from graphconvgeo_amd import sparse as gs

pytestmark = pytest.mark.gpu


def bow(n, f, dense_cols, density=0.3, per_row=12, seed=0):
    """Zipf-ish bag of words plus `dense_cols` columns present in `density` of the rows."""
    rng = np.random.default_rng(seed)
    rows = np.repeat(np.arange(n), per_row)
    cols = np.minimum(rng.zipf(1.3, size=n * per_row) + dense_cols, f - 1)
    r2, c2 = [], []
    for j in range(dense_cols):
        m = np.nonzero(rng.random(n) < density)[0]
        r2.append(m)
        c2.append(np.full(m.size, j))
    r = np.concatenate([rows] + r2)
    c = np.concatenate([cols] + c2)
    v = rng.random(r.size).astype(np.float32) + 0.05
    X = sps.csr_matrix((v, (r, c)), shape=(n, f), dtype=np.float32)
    X.sum_duplicates()
    X.sort_indices()
    return X


def check_close(Y, X, G):
    Y = Y.cpu().numpy().astype(np.float64)
    X64 = X.astype(np.float64)
    G64 = G.cpu().numpy().astype(np.float64)
    ref = X64.T @ G64
    bound = 1e-5 * (abs(X64).T @ np.abs(G64)) + 1e-30
    assert np.all(np.abs(Y - ref) <= bound), float((np.abs(Y - ref) / bound).max())


@pytest.mark.parametrize("K", [1, 37, 300])
def test_tmatmul_dense_column_split(monkeypatch, K):
    monkeypatch.setattr(gs, "HYBRID_MIN_ROWS", 1000)
    X = bow(20000, 3000, dense_cols=7, seed=K)
    A = gs.DeviceCSR.from_scipy(X, "cuda")
    G = torch.randn(20000, K, device="cuda")
    Y = A.tmatmul(G, mode="fast")
    cols, Xh, _ = A._dense_split
    counts = np.bincount(X.indices, minlength=X.shape[1])
    q = int((counts >= np.ceil(gs.HYBRID_MIN_DENSITY * X.shape[0])).sum())
    c = cols.cpu().numpy()
    # every qualifying column, topped up to a multiple of 64 with the next most frequent
    assert c.size == min((q + 63) // 64 * 64, gs.HYBRID_MAX_COLS) and q >= 7
    assert np.all(np.diff(c) > 0)
    rest = np.setdiff1d(np.arange(X.shape[1]), c)
    assert counts[c].min() >= counts[rest].max()
    check_close(Y, X, G)
    # the head block holds exactly X's head columns
    np.testing.assert_array_equal(Xh.cpu().numpy(), X[:, cols.cpu().numpy()].toarray())
    # ordered: bitwise the CSR(X^T) gather, no split
    Yo = A.tmatmul(G, mode="ordered")
    assert torch.equal(Yo, gs.spmm(A.transpose(), G, mode="ordered"))
    check_close(Yo, X, G)


def test_tmatmul_caps_dense_columns_at_the_most_frequent(monkeypatch):
    monkeypatch.setattr(gs, "HYBRID_MIN_ROWS", 1000)
    monkeypatch.setattr(gs, "HYBRID_MAX_COLS", 3)
    X = bow(8000, 500, dense_cols=6, seed=3)
    A = gs.DeviceCSR.from_scipy(X, "cuda")
    G = torch.randn(8000, 20, device="cuda")
    Y = A.tmatmul(G, mode="fast")
    cols = A._dense_split[0].cpu().numpy()
    counts = np.bincount(X.indices, minlength=500)
    top = np.sort(np.argsort(-counts, kind="stable")[:3])
    assert cols.size == 3 and set(counts[cols]) == set(counts[top])
    check_close(Y, X, G)


def test_tmatmul_without_dense_columns_is_the_gather(monkeypatch):
    monkeypatch.setattr(gs, "HYBRID_MIN_ROWS", 1000)
    rng = np.random.default_rng(5)
    X = sps.random(6000, 4000, density=0.002, format="csr", dtype=np.float32, random_state=rng)
    A = gs.DeviceCSR.from_scipy(X, "cuda")
    G = torch.randn(6000, 16, device="cuda")
    Y = A.tmatmul(G, mode="fast")
    assert A._dense_split is None
    assert torch.equal(Y, gs.spmm(A.transpose(), G, mode="fast"))


def test_tmatmul_auto_keeps_bitwise_when_rows_do_not_split(monkeypatch):
    """'auto' splits only when CSR(X^T) would run 'fast' (not bitwise) anyway."""
    monkeypatch.setattr(gs, "HYBRID_MIN_ROWS", 1000)
    X = bow(4000, 800, dense_cols=2, seed=9)
    A = gs.DeviceCSR.from_scipy(X, "cuda")
    G = torch.randn(4000, 8, device="cuda")
    T = A.transpose()
    Y = A.tmatmul(G, mode="auto")
    if T.max_row_nnz() * gs.TMATMUL_SPLIT_RATIO <= T.nnz:
        assert "_dense_split" not in A.__dict__
        assert torch.equal(Y, gs.spmm(T, G, mode="ordered"))
    else:
        assert A._dense_split is not None
    check_close(Y, X, G)
