"""GPU parity of the fused rectify backward (gcg_relu_backward_f32): g = gY where Y > 0 and
the bias gradient sum_rows(g) in one pass -- the gradient of rectify(H.Z + b1) that Theano
derives for mlpconv.py:75-77. The mask is bit-exact; the column sum is deterministic (fixed
block order) and within 1e-5 relative of the float64 sum."""
import numpy as np
import pytest
import torch

from graphconvgeo_amd import sparse as gs

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("M,K,ld", [(1, 1, 1), (7, 3, 3), (513, 64, 64), (1000, 255, 256),
                                    (5000, 300, 300), (4097, 1024, 1024), (700_001, 300, 300), (2000, 301, 304), (700, 301, 301),
                                    (1025, 20, 24)])
def test_relu_backward_matches_numpy(M, K, ld):
    rng = np.random.default_rng(M * 31 + K)
    gY = rng.standard_normal((M, ld)).astype(np.float32)
    Y = np.maximum(rng.standard_normal((M, ld)), 0).astype(np.float32)
    gd = torch.from_numpy(gY).cuda()[:, :K]
    Yd = torch.from_numpy(Y).cuda()[:, :K]
    g, db = gs.relu_backward(gd, Yd)
    ref = np.where(Y[:, :K] > 0, gY[:, :K], 0).astype(np.float32)
    np.testing.assert_array_equal(g.cpu().numpy(), ref)
    db_ref = ref.astype(np.float64).sum(0)
    np.testing.assert_allclose(db.cpu().numpy(), db_ref, rtol=1e-5,
                               atol=1e-5 * np.abs(ref).sum(0).max())
    g2, db2 = gs.relu_backward(gd, Yd)
    assert torch.equal(db, db2) and torch.equal(g, g2)


def test_relu_backward_in_place_and_no_bias():
    M, K = 3000, 128
    gY = torch.randn(M, K, device="cuda")
    Y = torch.relu(torch.randn(M, K, device="cuda"))
    ref = gY * (Y > 0)
    g, db = gs.relu_backward(gY, Y, out=gY, bias_grad=False)
    assert db is None and g.data_ptr() == gY.data_ptr()
    assert torch.equal(g, ref)


def test_relu_backward_empty():
    gY = torch.empty(0, 16, device="cuda")
    g, db = gs.relu_backward(gY, gY.clone())
    assert g.shape == (0, 16) and torch.equal(db, torch.zeros(16, device="cuda"))


@pytest.mark.parametrize("M,K,ld", [(1, 1, 1), (3, 5, 5), (777, 930, 932), (600_001, 300, 300),
                                    (4000, 1024, 1024), (9000, 301, 301)])
def test_column_sum_matches_float64(M, K, ld):
    rng = np.random.default_rng(M + K)
    X = rng.standard_normal((M, ld)).astype(np.float32)
    Xd = torch.from_numpy(X).cuda()[:, :K]
    s = gs.column_sum(Xd)
    ref = X[:, :K].astype(np.float64).sum(0)
    np.testing.assert_allclose(s.cpu().numpy(), ref, rtol=0,
                               atol=2e-6 * np.abs(X[:, :K]).sum(0).max() + 1e-7)
    assert torch.equal(s, gs.column_sum(Xd))  # deterministic


def _colsum_in_kernel_order(X):
    """numpy float32 restatement of the kernels' summation order (csr_ops.hip): blocks of rpb
    rows, wave w of a block adding rows w, w + 4, ... in order, the 4 waves combined
    ((0 + 1) + 2) + 3; then 16 streams over the block partials (stream s: blocks s, s + 16, ...)
    added 0..15 in order."""
    M, K = X.shape
    r = -(-M // 1024)
    rpb = max(512, (r + 3) // 4 * 4)
    nb = -(-M // rpb)
    part = np.zeros((nb, K), np.float32)
    for b in range(nb):
        r0, r1 = b * rpb, min(M, (b + 1) * rpb)
        acc = np.zeros((4, K), np.float32)
        for i in range(r0, r1):
            acc[(i - r0) % 4] += X[i]
        part[b] = ((acc[0] + acc[1]) + acc[2]) + acc[3]
    s = np.zeros((16, K), np.float32)
    for b in range(nb):
        s[b % 16] += part[b]
    t = s[0].copy()
    for i in range(1, 16):
        t += s[i]
    return t


@pytest.mark.parametrize("M,K,ld", [(20_000, 930, 960), (10_247, 300, 304), (9_000, 301, 301)])
def test_column_sums_follow_the_documented_order(M, K, ld):
    """Bitwise: the bias gradients are the fixed-order sums the kernels document (so a change
    of the finishing kernel's workgroup shape cannot move a bit)."""
    rng = np.random.default_rng(K)
    X = rng.standard_normal((M, ld)).astype(np.float32)
    Y = np.maximum(rng.standard_normal((M, ld)), 0).astype(np.float32)
    Xd = torch.from_numpy(X).cuda()[:, :K]
    np.testing.assert_array_equal(gs.column_sum(Xd).cpu().numpy(), _colsum_in_kernel_order(X[:, :K]))
    _, db = gs.relu_backward(Xd, torch.from_numpy(Y).cuda()[:, :K])
    masked = np.where(Y[:, :K] > 0, X[:, :K], np.float32(0))
    np.testing.assert_array_equal(db.cpu().numpy(), _colsum_in_kernel_order(masked))
