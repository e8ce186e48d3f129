"""GPU parity of the MFMA dense kernels (csrc/dense.hip): the output layer's T.dot(h, W) + b
(mlpconv.py:88-93), softmax / categorical cross-entropy / accuracy (mlpconv.py:227-253)
and their gradients, against float64 restatements (oracle.gcn_oracle.softmax_xent_f64).

Tolerances (fp32 MFMA = exact f32 products, f32 accumulation in a permuted k order):
  GEMM        |C - C64| <= 2e-6 * (|A| @ |B|) + 1e-30   (a few ulps of the absolute sum)
  softmax/CE  |.| <= 1e-5 (probabilities / gradients <= 1 in magnitude, K <= 1024)
"""
import numpy as np
import pytest
import torch

from graphconvgeo_amd import dense
from graphconvgeo_amd.sparse import empty_dense
from oracle import gcn_oracle as O

pytestmark = pytest.mark.gpu


def _rand(shape, seed, scale=1.0):
    return (np.random.default_rng(seed).standard_normal(shape) * scale).astype(np.float32)


def _check_gemm(C, A, B, bias=None, relu=False):
    C64 = A.astype(np.float64) @ B.astype(np.float64)
    if bias is not None:
        C64 = C64 + bias.astype(np.float64)
    if relu:
        C64 = np.maximum(C64, 0)
    bound = 2e-6 * (np.abs(A).astype(np.float64) @ np.abs(B).astype(np.float64)
                    + (0 if bias is None else np.abs(bias))) + 1e-30
    err = np.abs(C.astype(np.float64) - C64)
    assert (err <= bound).all(), f"max err {err.max()} (bound at worst {bound.ravel()[err.argmax()]})"


def _padded(W, dev, transpose=False):
    return dense._WeightCache().get(torch.from_numpy(W).to(dev), transpose)


@pytest.mark.parametrize("M,K,N", [(1, 1, 1), (5, 3, 7), (33, 16, 64), (64, 17, 65),
                                   (100, 64, 129), (257, 300, 256), (130, 300, 300),
                                   (70, 300, 321), (96, 300, 930), (40, 930, 300),
                                   (31, 65, 1024), (50, 40, 1500), (300, 129, 4)])
def test_gemm_vs_float64(cuda, M, K, N):
    A, B = _rand((M, K), 1), _rand((K, N), 2)
    C = dense.gemm(torch.from_numpy(A).to(cuda), _padded(B, cuda)).cpu().numpy()
    _check_gemm(C, A, B)


def test_gemm_bias_relu_and_strided(cuda):
    M, K, N = 200, 300, 930
    A, B, b = _rand((M, K), 3), _rand((K, N), 4), _rand((N,), 5)
    At = torch.from_numpy(A).to(cuda)
    bt = torch.from_numpy(b).to(cuda)
    C = dense.gemm(At, _padded(B, cuda), bias=bt, act="relu").cpu().numpy()
    _check_gemm(C, A, B, bias=b, relu=True)
    # A with a leading dimension that is not a multiple of 4 is re-laid out, same result
    big = torch.zeros((M, K + 3), device=cuda)
    big[:, :K] = At
    C2 = dense.gemm(big[:, :K], _padded(B, cuda), bias=bt, act="relu").cpu().numpy()
    assert np.array_equal(C, C2)
    # output into a caller-owned padded buffer
    out = empty_dense(M, N, cuda)
    dense.gemm(At, _padded(B, cuda), bias=bt, act="relu", out=out)
    assert np.array_equal(out.cpu().numpy(), C)


def test_gemm_exact_integer_layout(cuda):
    """Small-integer operands: every product and sum is exact in f32, so any lane/row/column
    mix-up shows as an exact mismatch (asymmetric B)."""
    rng = np.random.default_rng(7)
    M, K, N = 77, 45, 330
    A = rng.integers(-3, 4, (M, K)).astype(np.float32)
    B = rng.integers(-3, 4, (K, N)).astype(np.float32)
    B[0, :] = np.arange(N)  # asymmetric
    C = dense.gemm(torch.from_numpy(A).to(cuda), _padded(B, cuda)).cpu().numpy()
    assert np.array_equal(C, (A.astype(np.int64) @ B.astype(np.int64)).astype(np.float32))


def test_gemm_rejects_bad_operands(cuda):
    A = torch.randn(8, 12, device=cuda)
    with pytest.raises(ValueError):
        dense.gemm(A, torch.randn(12, 10, device=cuda))  # ld 10 < round4(10) = 12
    with pytest.raises(ValueError):
        dense.gemm(A, torch.randn(11, 12, device=cuda))
    with pytest.raises(ValueError):
        dense.gemm(A.cpu(), torch.randn(12, 12))


@pytest.mark.parametrize("M,K,N", [(1, 4, 2), (37, 16, 129), (300, 300, 256), (513, 300, 930),
                                   (64, 65, 1024), (20, 3, 61), (40, 50, 300), (33, 70, 700),
                                   (20, 16, 700), (9, 4, 520), (70, 300, 600)])
@pytest.mark.parametrize("math", ["bf16x6", "f32"])
def test_fused_softmax_xent_vs_float64(cuda, M, K, N, math, monkeypatch):
    """The fused output layer, on the bf16 matrix cores (gemm_fused6_kernel, the default) and on
    the f32 MFMA (math GCG_MATH_F32, gemm_kernel): loss, gradient, hits, probabilities."""
    monkeypatch.setattr(dense, "FUSED_MATH", math)
    P, W, b = _rand((M, K), 11, 0.3), _rand((K, N), 12, 0.3), _rand((N,), 13)
    y = np.random.default_rng(14).integers(0, N, M).astype(np.int32)
    proj = dense.Projection()
    Pt, Wt, bt = (torch.from_numpy(v).to(cuda) for v in (P, W, b))
    yt = torch.from_numpy(y).to(cuda)
    G = empty_dense(M, N, cuda)
    loss = torch.empty(M, device=cuda)
    hits = torch.empty(M, device=cuda)
    dense._fused(Pt, proj.fwd.get(Wt, False), bt, yt, 1.0 / M, None, G, loss, hits)
    logits64 = P.astype(np.float64) @ W.astype(np.float64) + b
    P64, loss64, hits64, G64 = O.softmax_xent_f64(logits64, y)
    assert np.abs(loss.cpu().numpy() - loss64).max() < 1e-5
    assert np.abs(G.cpu().numpy() - G64).max() < 1e-5 / M + 1e-7
    # hits: compare where the top-2 margin is clearly above f32 rounding
    srt = np.sort(logits64, axis=1)
    clear = (srt[:, -1] - srt[:, -2] if N > 1 else np.ones(M)) > 1e-4
    assert np.array_equal(hits.cpu().numpy()[clear], hits64[clear])
    probs = proj.probabilities(Pt, Wt, bt).cpu().numpy()
    assert np.abs(probs - P64).max() < 1e-5
    # loss-only evaluation (no gradient written)
    loss2 = torch.empty(M, device=cuda)
    dense._fused(Pt, proj.fwd.get(Wt, False), bt, yt, 1.0, None, None, loss2, None)
    assert torch.equal(loss, loss2)


@pytest.mark.parametrize("N", [129, 930])
@pytest.mark.parametrize("math", ["bf16x6", "f32"])
def test_fused_labels_outside_classes(cuda, N, math, monkeypatch):
    """A label outside [0, N) (-1, N, N + 7; the C-ABI does not check labels on the host): that
    row's loss is NaN, its hit 0, and its gradient row the probabilities times scale (no onehot
    subtracted); every other row as with valid labels. Both maths, the 64-row tile at N = 930."""
    monkeypatch.setattr(dense, "FUSED_MATH", math)
    M, K = 70, 33
    P, W, b = _rand((M, K), 61, 0.3), _rand((K, N), 62, 0.3), _rand((N,), 63)
    y = np.random.default_rng(64).integers(0, N, M).astype(np.int32)
    bad = np.array([3, 17, 40, 69])
    y[bad] = [-1, N, N + 7, -5]
    ok = np.ones(M, bool)
    ok[bad] = False
    Pt, Wt, bt = (torch.from_numpy(v).to(cuda) for v in (P, W, b))
    yt = torch.from_numpy(y).to(cuda)
    G = empty_dense(M, N, cuda)
    loss, hits = torch.empty(M, device=cuda), torch.empty(M, device=cuda)
    dense._fused(Pt, dense.Projection().fwd.get(Wt, False), bt, yt, 1.0 / M, None, G, loss, hits)
    logits64 = P.astype(np.float64) @ W.astype(np.float64) + b
    P64, loss64, hits64, G64 = O.softmax_xent_f64(logits64, np.where(ok, y, 0))
    lo, hi, Gc = loss.cpu().numpy(), hits.cpu().numpy(), G.cpu().numpy()
    assert np.isnan(lo[bad]).all() and (hi[bad] == 0).all()
    assert np.abs(Gc[bad] - P64[bad] / M).max() < 1e-5 / M + 1e-7
    assert np.abs(lo[ok] - loss64[ok]).max() < 1e-5
    assert np.abs(Gc[ok] - G64[ok]).max() < 1e-5 / M + 1e-7
    srt = np.sort(logits64, axis=1)
    clear = ok & ((srt[:, -1] - srt[:, -2]) > 1e-4)
    assert np.array_equal(hi[clear], hits64[clear])


@pytest.mark.parametrize("M,K,N", [(37, 16, 129), (513, 300, 930), (20, 3, 61), (9, 4, 522),
                                   (40, 50, 300), (70, 300, 600)])
@pytest.mark.parametrize("math,presplit", [("bf16x6", True), ("bf16x6", False), ("f32", True)])
def test_fused_nan_weight_padding_never_leaks(cuda, M, K, N, math, presplit, monkeypatch):
    """W's padding columns [N, ldw) may hold anything (gcg_spmm.h): NaN there must not reach
    the softmax sum, the loss or the gradient -- bitwise the zero-padded result. presplit False:
    the bf16x6 form that splits W in registers and so reads its padding columns; its non-finite
    check looks at columns < N only, so the NaN does not send the tile down the f32 path
     -- which would change its bits."""
    monkeypatch.setattr(dense, "FUSED_MATH", math)
    monkeypatch.setattr(dense, "FUSED_PRESPLIT", presplit)
    P, W, b = _rand((M, K), 31, 0.3), _rand((K, N), 32, 0.3), _rand((N,), 33)
    y = np.random.default_rng(34).integers(0, N, M).astype(np.int32)
    Pt, Wt, bt = (torch.from_numpy(v).to(cuda) for v in (P, W, b))
    yt = torch.from_numpy(y).to(cuda)
    ldw = (N + 3) // 4 * 4 + 4
    outs = []
    for fill in (0.0, float("nan"), float("inf")):
        Wp = torch.full((K, ldw), fill, device=cuda)
        Wp[:, :N] = Wt
        G = empty_dense(M, N, cuda)
        loss, hits = torch.empty(M, device=cuda), torch.empty(M, device=cuda)
        dense._fused(Pt, Wp[:, :N], bt, yt, 1.0 / M, None, G, loss, hits)
        probs = empty_dense(M, N, cuda)
        dense._fused(Pt, Wp[:, :N], bt, None, 1.0, None, probs, torch.empty(M, device=cuda), None)
        outs.append((G, loss, hits, probs))
    assert torch.isfinite(outs[0][0]).all() and torch.isfinite(outs[0][1]).all()
    for o in outs[1:]:
        for a, ref in zip(o, outs[0]):
            assert torch.equal(a, ref)


@pytest.mark.parametrize("M,K,N", [(37, 16, 129), (300, 300, 256), (513, 300, 930), (70, 33, 1024),
                                   (40, 50, 300), (33, 70, 700), (65, 17, 900)])
def test_fused_split_pingpong_bitwise(cuda, M, K, N):
    """The f32 MFMA fused layer's tiles 1..5 (the B register set split into 0 / 2 / 4 / 8 / 16
    rotating parts) only reorder MFMAs between distinct accumulators: gradient, loss and hits
    bitwise equal to tile 0 (the default)."""
    assert dense.tile_count("fused", "f32") == 5
    P, W, b = _rand((M, K), 21, 0.3), _rand((K, N), 22, 0.3), _rand((N,), 23)
    y = np.random.default_rng(24).integers(0, N, M).astype(np.int32)
    Pt, Wt, bt = (torch.from_numpy(v).to(cuda) for v in (P, W, b))
    yt = torch.from_numpy(y).to(cuda)
    Wp = dense.Projection().fwd.get(Wt, False)
    outs = []
    for tile in range(6):
        G = empty_dense(M, N, cuda)
        loss, hits = torch.empty(M, device=cuda), torch.empty(M, device=cuda)
        dense._fused(Pt, Wp, bt, yt, 1.0 / M, None, G, loss, hits, math="f32", tile=tile)
        outs.append((G, loss, hits))
    for G, loss, hits in outs[1:]:
        assert torch.equal(G, outs[0][0]) and torch.equal(loss, outs[0][1])
        assert torch.equal(hits, outs[0][2])


@pytest.mark.parametrize("M,K,N", [(37, 16, 129), (513, 300, 930), (70, 33, 1024), (65, 17, 600),
                                   (9, 4, 61), (5, 7, 801), (128, 64, 1021), (100, 48, 930),
                                   (100, 49, 930)])
def test_fused6_row_bands_bitwise(cuda, M, K, N, monkeypatch):
    """gemm_fused6_kernel's forms (math GCG_MATH_BF16X6): the weight split in every workgroup's
    registers (no workspace; dense.FUSED_PRESPLIT off), the weight's planes pre-split into the
    workspace on the 32-row 4-wave tile (tile 1) -- the same products in the same order: bitwise
    equal (gradient, loss, hits, probabilities), rows past M included -- and on the 64-row 8-wave
    tile (tile 2; tile 0 picks it at N > 768), whose row sums run over 8 column waves (another
    association): within f32 rounding, the same hits. Tile 3 (tile 0's shape with the A chunk
    split cooperatively into LDS planes) is bitwise the form of that shape."""
    assert dense.tile_count("fused", "bf16x6") == 3
    P, W, b = _rand((M, K), 51, 0.3), _rand((K, N), 52, 0.3), _rand((N,), 53)
    y = np.random.default_rng(54).integers(0, N, M).astype(np.int32)
    Pt, Wt, bt = (torch.from_numpy(v).to(cuda) for v in (P, W, b))
    yt = torch.from_numpy(y).to(cuda)
    Wp = dense.Projection().fwd.get(Wt, False)

    def run(presplit, tile=0):
        monkeypatch.setattr(dense, "FUSED_PRESPLIT", presplit)
        G = empty_dense(M, N, cuda)
        loss, hits = torch.empty(M, device=cuda), torch.empty(M, device=cuda)
        dense._fused(Pt, Wp, bt, yt, 1.0 / M, None, G, loss, hits, math="bf16x6", tile=tile)
        probs = empty_dense(M, N, cuda)
        dense._fused(Pt, Wp, bt, None, 1.0, None, probs, torch.empty(M, device=cuda), None,
                     math="bf16x6", tile=tile)
        return G, loss, hits, probs

    ref = run(False)
    for a, r in zip(run(True, tile=1), ref):
        assert torch.equal(a, r)
    wide = [run(True)] + ([run(True, tile=2)] if N > 768 else [])
    if N <= 768:  # tile 0 is the 32-row form there
        for a, r in zip(wide[0], ref):
            assert torch.equal(a, r)
        from graphconvgeo_amd._native import NativeError
        with pytest.raises(NativeError):
            run(True, tile=2)  # the 64-row tile needs N > 768
    # tile 3: tile 0's shape with the cooperative A split -- bitwise the 32-row form at N <= 768,
    # the 64-row one above
    for a, r in zip(run(True, tile=3), ref if N <= 768 else wide[1]):
        assert torch.equal(a, r)
    for G2, l2, h2, p2 in wide:
        assert torch.equal(h2, ref[2])
        assert float((l2 - ref[1]).abs().max()) < 1e-5
        assert float((G2 - ref[0]).abs().max()) < 1e-6 / M + 1e-9
        assert float((p2 - ref[3]).abs().max()) < 1e-6


def test_rows_softmax_xent_vs_float64(cuda):
    for M, N in [(1, 1), (9, 3), (1000, 930), (257, 256), (33, 4096), (5, 1025)]:
        L = _rand((M, N), M + N, 3.0)
        y = np.random.default_rng(M).integers(0, N, M).astype(np.int32)
        Lt = torch.from_numpy(L).to(cuda)
        P64, loss64, hits64, G64 = O.softmax_xent_f64(L, y)
        loss, acc = dense.softmax_xent(Lt, torch.from_numpy(y).to(cuda))
        assert abs(float(loss) - loss64.mean()) < 1e-5 * max(1.0, abs(loss64.mean()))
        assert abs(float(acc) - hits64.mean()) < 1.5 / M
        probs = dense.softmax(Lt).cpu().numpy()
        assert np.abs(probs - P64).max() < 1e-5


def test_project_xent_autograd_vs_float64(cuda):
    M, K, N = 400, 300, 129
    P, W, b = _rand((M, K), 21, 0.2), _rand((K, N), 22, 0.2), _rand((N,), 23, 0.1)
    y = np.random.default_rng(24).integers(0, N, M)
    Pt = torch.from_numpy(P).to(cuda).requires_grad_()
    Wt = torch.from_numpy(W).to(cuda).requires_grad_()
    bt = torch.from_numpy(b).to(cuda).requires_grad_()
    loss, acc = dense.project_softmax_xent(Pt, Wt, bt, torch.from_numpy(y).to(cuda))
    (loss * 2.5).backward()  # upstream gradient != 1 goes through the folded scale
    logits64 = P.astype(np.float64) @ W + b
    _, loss64, hits64, G64 = O.softmax_xent_f64(logits64, y)
    G64 = G64 * 2.5
    assert abs(float(loss.detach()) - loss64.mean()) < 1e-5
    assert np.abs(Pt.grad.cpu().numpy() - G64 @ W.T.astype(np.float64)).max() < 1e-6
    assert np.abs(Wt.grad.cpu().numpy() - P.T.astype(np.float64) @ G64).max() < 1e-5
    assert np.abs(bt.grad.cpu().numpy() - G64.sum(0)).max() < 1e-5


def test_rows_xent_autograd_and_matmul_autograd(cuda):
    M, K, N = 300, 64, 200
    A, W, b = _rand((M, K), 31, 0.3), _rand((K, N), 32, 0.3), _rand((N,), 33, 0.1)
    y = np.random.default_rng(34).integers(0, N, M)
    proj = dense.Projection()
    At = torch.from_numpy(A).to(cuda).requires_grad_()
    Wt = torch.from_numpy(W).to(cuda).requires_grad_()
    bt = torch.from_numpy(b).to(cuda).requires_grad_()
    logits = proj.matmul(At, Wt, bt)
    loss, _ = dense.softmax_xent(logits, torch.from_numpy(y).to(cuda))
    (0.5 * loss).backward()
    _, loss64, _, G64 = O.softmax_xent_f64(A.astype(np.float64) @ W + b, y)
    G64 *= 0.5
    assert abs(float(loss.detach()) - loss64.mean()) < 1e-5
    assert np.abs(At.grad.cpu().numpy() - G64 @ W.T.astype(np.float64)).max() < 1e-6
    assert np.abs(Wt.grad.cpu().numpy() - A.T.astype(np.float64) @ G64).max() < 1e-6
    assert np.abs(bt.grad.cpu().numpy() - G64.sum(0)).max() < 1e-6


def test_fused_rejects_too_many_classes(cuda):
    with pytest.raises(ValueError):
        dense.project_softmax_xent(torch.randn(4, 8, device=cuda), torch.randn(8, 1025, device=cuda),
                                   None, torch.zeros(4, dtype=torch.int64, device=cuda))


@pytest.mark.parametrize("R,M,N", [(1, 1, 1), (7, 3, 5), (100, 64, 129), (4097, 300, 930),
                                   (20000, 48, 60), (3, 320, 1024), (0, 4, 4)])
def test_gemm_tn_vs_float64(cuda, R, M, N):
    """Weight-gradient GEMM C = A^T . B (split-K MFMA, partials summed in split order)."""
    A, B = _rand((R, M), 41, 0.5), _rand((R, N), 42, 0.5)
    At, Bt = torch.from_numpy(A).to(cuda), torch.from_numpy(B).to(cuda)
    C = dense.gemm_tn(At, Bt).cpu().numpy()
    _check_gemm(C, A.T.copy(), B)
    C2 = dense.gemm_tn(At, Bt).cpu().numpy()
    assert np.array_equal(C, C2)  # deterministic
    sc = torch.tensor(2.5, device=cuda)
    C3 = dense.gemm_tn(At, Bt, scale=sc).cpu().numpy()
    assert np.array_equal(C3, (C * np.float32(2.5)))


@pytest.mark.parametrize("tile", [1, 2, 3, 4, 5, 6, 7])
@pytest.mark.parametrize("R,M,N", [(4097, 300, 930), (70001, 256, 300), (513, 70, 129), (5, 3, 200)])
def test_gemm_tn_layouts_vs_float64(cuda, R, M, N, tile):
    """Every split-K wave layout (gcg_gemm_tn tiles 1..7: workgroup tiles WM = 1, per-wave tiles
    WM = 0 -- the default family -- and waves stacked along M) against float64, with ragged R
    (steps that end inside a split read zeros through the buffer range check), M and N off the
    tiles."""
    assert dense.tile_count("gemm_tn") == 7 and dense.tile_count("gemm_tn", "bf16x6") == 0
    A, B = _rand((R, M), 45, 0.5), _rand((R, N), 46, 0.5)
    At, Bt = torch.from_numpy(A).to(cuda), torch.from_numpy(B).to(cuda)
    C = dense.gemm_tn(At, Bt, tile=tile).cpu().numpy()
    _check_gemm(C, A.T.copy(), B)
    assert np.array_equal(C, dense.gemm_tn(At, Bt, tile=tile).cpu().numpy())  # deterministic


def test_gemm_tn_strided_views(cuda):
    R, M, N = 3000, 300, 930
    A, B = _rand((R, M), 43), _rand((R, N), 44)
    Bbuf = empty_dense(R, N, cuda)  # ld 960, the layout of the fused kernel's gradient
    Bbuf.copy_(torch.from_numpy(B))
    C = dense.gemm_tn(torch.from_numpy(A).to(cuda), Bbuf).cpu().numpy()
    _check_gemm(C, A.T.copy(), B)


def _weight_grads(cuda, side: bool, shared_w: bool):
    """W used by project_softmax_xent and (optionally) a second matmul; gradients accumulate."""
    old = dense.SIDE_STREAM_WEIGHT_GRADS
    dense.SIDE_STREAM_WEIGHT_GRADS = side
    try:
        M, K, N = 3000, 300, 129
        P, W, b = _rand((M, K), 41, 0.2), _rand((K, N), 42, 0.2), _rand((N,), 43, 0.1)
        y = torch.from_numpy(np.random.default_rng(44).integers(0, N, M)).to(cuda)
        Pt = torch.from_numpy(P).to(cuda).requires_grad_()
        Wt = torch.from_numpy(W).to(cuda).requires_grad_()
        bt = torch.from_numpy(b).to(cuda).requires_grad_()
        Wt.grad = torch.full_like(Wt, 0.25)  # accumulate into an existing gradient
        loss, _ = dense.project_softmax_xent(Pt, Wt, bt, y)
        if shared_w:
            loss = loss + dense.matmul(Pt * 1.5, Wt).square().mean()
        (loss * 3.0).backward()
        torch.cuda.synchronize()
        return Pt.grad.clone(), Wt.grad.clone(), bt.grad.clone()
    finally:
        dense.SIDE_STREAM_WEIGHT_GRADS = old


@pytest.mark.parametrize("shared_w", [False, True])
def test_side_stream_weight_grads_equal_inline(cuda, shared_w):
    """The weight gradient computed on the side stream (overlapping the rest of the backward)
    is bitwise the inline one, also when W feeds two products and W.grad already exists."""
    a = _weight_grads(cuda, True, shared_w)
    b = _weight_grads(cuda, False, shared_w)
    for x, y in zip(a, b):
        assert torch.equal(x, y)


@pytest.mark.parametrize("M,K,N", [(1, 1, 1), (65, 17, 5), (129, 300, 300), (200, 33, 320),
                                   (257, 64, 321), (130, 300, 512), (300, 300, 930),
                                   (77, 40, 1024), (100, 20, 1500), (64, 930, 300)])
def test_lds_b_gemm_equals_register_b_gemm(cuda, M, K, N):
    """The plain products' default tile (B staged through LDS, gemm_bl_kernel) accumulates in
    the same k order as tile 1 (gemm_kernel, B straight to registers): bitwise equal, bias +
    rectify included."""
    A, B, bias = _rand((M, K), M + 1), _rand((K, N), N + 2), _rand((N,), 3)
    At = torch.from_numpy(A).to(cuda)
    Bt = _padded(B, cuda)
    bt = torch.from_numpy(bias).to(cuda)
    outs = []
    for tile in (0, 1):
        outs.append((dense.gemm(At, Bt, tile=tile),
                     dense.gemm(At, Bt, bias=bt, act="relu", tile=tile)))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    _check_gemm(outs[0][1].cpu().numpy(), A, B, bias, relu=True)


@pytest.mark.parametrize("M,K,N", [(1, 1, 1), (5, 3, 7), (33, 16, 64), (64, 17, 65),
                                   (129, 31, 63), (257, 300, 256), (130, 300, 300),
                                   (70, 300, 321), (96, 300, 930), (300, 930, 300),
                                   (31, 65, 1024), (50, 40, 1500), (300, 129, 4),
                                   (1000, 256, 300), (517, 33, 930)])
@pytest.mark.parametrize("math", dense.NT_MATHS)
def test_gemm_nt_vs_float64(cuda, M, K, N, math):
    """gcg_gemm_nt_f32 (LDS-DMA staged, both operands k-contiguous): C = A . Bt^T; and the same
    product on the bf16 matrix cores (gcg_gemm_nt_f32_bf16x6, pre-split weight planes or both
    operands split in the loop) within the same float64 bar."""
    A, B = _rand((M, K), 11), _rand((K, N), 12)
    Bt = _padded(B, cuda, transpose=True)  # N x round4(K)
    C = dense.gemm_nt(torch.from_numpy(A).to(cuda), Bt, math=math).cpu().numpy()
    _check_gemm(C, A, B)


@pytest.mark.parametrize("tile", list(range(11)))
def test_gemm_nt_tile_variants(cuda, tile):
    """Every f32 NT tile (gcg_gemm_nt math GCG_MATH_F32, tiles 0..10) on ragged M / N / K, bias +
    relu: within the float64 bar and bitwise equal to tile 0 (the same k order)."""
    assert dense.tile_count("gemm_nt", "f32") == 10
    M, K, N = 333, 301, 133
    A, B, b = _rand((M, K), 13), _rand((K, N), 14), _rand((N,), 15)
    At, Bt, bt = torch.from_numpy(A).to(cuda), _padded(B, cuda, transpose=True), torch.from_numpy(b).to(cuda)
    C = dense.gemm_nt(At, Bt, bias=bt, act="relu", math="f32", tile=tile)
    _check_gemm(C.cpu().numpy(), A, B, bias=b, relu=True)
    assert torch.equal(C, dense.gemm_nt(At, Bt, bias=bt, act="relu", math="f32"))


@pytest.mark.parametrize("M,K,N", [(333, 301, 133), (1000, 300, 930), (517, 930, 300),
                                   (70, 33, 65), (1, 5, 3), (130, 48, 77), (131, 49, 77),
                                   (300, 600, 600)])
def test_gemm_nt_bf16x6_tiles_bitwise(cuda, M, K, N):
    """Every bf16x6 tile (gcg_gemm_nt math GCG_MATH_BF16X6, tiles 0..9: A in registers or through
    LDS, the weight planes read from LDS one slot ahead or not) and the in-loop split of both operands accumulate the same six plane products in the
    same order: bitwise equal to each other, with bias + relu, ragged M / N / K; within the
    float64 bar. The K tail is packed (mfma6) when the last chunk holds <= 16 k (K = 48: 16,
    K = 49: 17 -- not packed); tile 0 at K > 512 splits N ragged where that pads less (N = 300:
    192 + 128 columns; N = 600: 576 + 64)."""
    assert dense.tile_count("gemm_nt", "bf16x6") == 9
    A, B, b = _rand((M, K), 13), _rand((K, N), 14), _rand((N,), 15)
    At, Bt = torch.from_numpy(A).to(cuda), _padded(B, cuda, transpose=True)
    bt = torch.from_numpy(b).to(cuda)
    ref = dense.gemm_nt(At, Bt, bias=bt, act="relu", math="bf16x6_inloop")
    _check_gemm(ref.cpu().numpy(), A, B, bias=b, relu=True)
    for tile in range(10):
        C = dense.gemm_nt(At, Bt, bias=bt, act="relu", math="bf16x6", tile=tile)
        assert torch.equal(C, ref), tile


def test_gemm_nt_bf16x6_error_at_most_f32s(cuda):
    """The bf16x6 products are f32-accurate: on 4096 x 300 x 930 with operands spanning six
    decades (sign-mixed, log-uniform magnitudes), the largest error against float64 relative to
    sum_k |a||b| is within 1.25 x the f32 MFMA kernel's, and below 2^-20."""
    rng = np.random.default_rng(40)
    M, K, N = 4096, 300, 930
    A = (rng.choice([-1.0, 1.0], (M, K)) * 10.0 ** rng.uniform(-3, 3, (M, K))).astype(np.float32)
    B = (rng.choice([-1.0, 1.0], (K, N)) * 10.0 ** rng.uniform(-3, 3, (K, N))).astype(np.float32)
    At, Bt = torch.from_numpy(A).to(cuda), _padded(B, cuda, transpose=True)
    C64 = A.astype(np.float64) @ B.astype(np.float64)
    scale = np.abs(A).astype(np.float64) @ np.abs(B).astype(np.float64)
    rel = {}
    for math in ("f32", "bf16x6"):
        C = dense.gemm_nt(At, Bt, math=math).cpu().numpy().astype(np.float64)
        rel[math] = float((np.abs(C - C64) / scale).max())
    assert rel["bf16x6"] <= 1.25 * rel["f32"] and rel["bf16x6"] < 2.0 ** -20, rel


def test_gemm_nt_bf16x6_nan_propagates(cuda):
    """A NaN operand element reaches exactly the outputs whose dot product it enters."""
    M, K, N = 64, 100, 70
    A, B = _rand((M, K), 41), _rand((K, N), 42)
    A[5, 17] = np.nan
    B[33, 9] = np.nan
    for math in ("bf16x6", "bf16x6_inloop"):
        C = dense.gemm_nt(torch.from_numpy(A).to(cuda), _padded(B, cuda, transpose=True),
                          math=math).cpu().numpy()
        bad = np.zeros((M, N), bool)
        bad[5, :] = True
        bad[:, 9] = True
        assert np.array_equal(np.isnan(C), bad), math


@pytest.mark.parametrize("math", dense.NT_MATHS)
@pytest.mark.parametrize("tile", [0, 2, 5])
def test_gemm_nt_padding_never_leaks(cuda, math, tile):
    """The k tail is zeroed in the fragments: NaN in the operands' padding columns (k >= K, inside
    the row stride) and in rows past M / N must not reach C (bf16x6 tiles 2 / 5: A in
    registers 128 x 128, A through LDS 128 x 64; f32 tiles 2 / 5: PF, 128 x 128)."""
    if tile and math == "bf16x6_inloop":
        pytest.skip("the in-loop split has one tile")
    M, K, N = 200, 298, 70
    A, B = _rand((M, K), 16), _rand((K, N), 17)
    Ap = torch.full((M, 300), float("nan"), device=cuda)
    Ap[:, :K] = torch.from_numpy(A).to(cuda)
    Btp = torch.full((N, 300), float("nan"), device=cuda)
    Btp[:, :K] = torch.from_numpy(B.T.copy()).to(cuda)
    C = dense.gemm_nt(Ap[:, :K], Btp[:, :K], math=math, tile=tile).cpu().numpy()
    assert np.isfinite(C).all()
    _check_gemm(C, A, B)
    # bitwise the zero-padded product: the bf16x6 tiles' non-finite check looks at in-range
    # elements only, so NaN padding never sends an edge tile down the f32 path
    Ap.nan_to_num_(0.0)
    Btp.nan_to_num_(0.0)
    C0 = dense.gemm_nt(Ap[:, :K], Btp[:, :K], math=math, tile=tile).cpu().numpy()
    assert np.array_equal(C, C0)


def test_matmul_autograd_on_nt_kernels(cuda):
    """dense.matmul (T.dot(h, W) + b, mlpconv.py:88-93): forward, dA = g . W^T and dW, db."""
    M, K, N = 700, 300, 129
    A, W, b = _rand((M, K), 18), _rand((K, N), 19, 0.1), _rand((N,), 20)
    G = _rand((M, N), 21)
    At = torch.from_numpy(A).to(cuda).requires_grad_()
    Wt = torch.nn.Parameter(torch.from_numpy(W).to(cuda))
    bt = torch.nn.Parameter(torch.from_numpy(b).to(cuda))
    C = dense.matmul(At, Wt, bt)
    (C * torch.from_numpy(G).to(cuda)).sum().backward()
    _check_gemm(C.detach().cpu().numpy(), A, W, bias=b)
    _check_gemm(At.grad.cpu().numpy(), G, W.T.copy())
    _check_gemm(Wt.grad.cpu().numpy(), A.T.copy(), G)
    assert np.abs(bt.grad.cpu().numpy() - G.astype(np.float64).sum(0)).max() < 1e-4
    # the weight moves in place (Adam): the cached transposed copy must follow
    with torch.no_grad():
        Wt.mul_(2.0)
    C2 = dense.matmul(At.detach(), Wt, bt)
    _check_gemm(C2.detach().cpu().numpy(), A, 2 * W, bias=b)


def test_l1l2_penalty_vs_float64(cuda):
    """MLPCONV's weight penalty (mlpconv.py:235-243) on the HIP reduction + gradient kernels:
    value within 1e-6 relative of float64, deterministic (bitwise equal across calls), gradient
    s * (l1 sgn(W) + 2 l2 W) with sgn(0) = 0 and the upstream gradient s applied."""
    W2 = _rand((300, 129), 30, 0.05)
    W1 = _rand((1000, 300), 31, 0.05)
    W1[0, :7] = 0.0  # Theano's grad of abs is 0 at 0
    coefs = [(2.5e-5, 2.5e-5), (1e-4, 3e-5)]
    Ws = [torch.nn.Parameter(torch.from_numpy(W).to(cuda)) for W in (W2, W1)]
    pen = dense.l1l2_penalty(Ws, coefs)
    ref = sum(l1 * np.abs(W.astype(np.float64)).sum() + l2 * (W.astype(np.float64) ** 2).sum()
              for W, (l1, l2) in zip((W2, W1), coefs))
    assert abs(float(pen.detach()) - ref) <= 1e-6 * ref
    assert float(dense.l1l2_penalty(Ws, coefs).detach()) == float(pen.detach())
    (pen * 3.0).backward()
    for W, Wt, (l1, l2) in zip((W2, W1), Ws, coefs):
        g64 = 3.0 * (l1 * np.sign(W.astype(np.float64)) + 2 * l2 * W.astype(np.float64))
        assert np.abs(Wt.grad.cpu().numpy() - g64).max() <= 1e-6 * np.abs(g64).max()
    assert (Ws[1].grad[0, :7] == 0).all()
    with torch.no_grad():
        assert float(dense.l1l2_penalty([Ws[0]], coefs[:1])) > 0


@pytest.mark.parametrize("M,K,N", [(37, 16, 129), (513, 300, 930), (40, 50, 300)])
def test_weighted_softmax_xent_vs_float64(cuda, M, K, N):
    """Row weights (target multiplicities, gcg_*_softmax_xent_weighted_f32): row i's loss, hit
    and gradient row times w_i, in the fused layer (train and evaluation forms) and the row
    kernel; all-ones weights are bitwise the unweighted kernels."""
    P, W, b = _rand((M, K), 41, 0.3), _rand((K, N), 42, 0.3), _rand((N,), 43)
    y = np.random.default_rng(44).integers(0, N, M).astype(np.int32)
    w = np.random.default_rng(45).integers(1, 5, M).astype(np.float32)
    Pt, Wt, bt = (torch.from_numpy(v).to(cuda) for v in (P, W, b))
    yt, wt = torch.from_numpy(y).to(cuda), torch.from_numpy(w).to(cuda)
    Wp = dense.Projection().fwd.get(Wt, False)
    T = float(w.sum())
    logits64 = P.astype(np.float64) @ W.astype(np.float64) + b
    _P64, loss64, hits64, G64 = O.softmax_xent_f64(logits64, y, scale=1.0 / T)
    G = empty_dense(M, N, cuda)
    loss, hits = torch.empty(M, device=cuda), torch.empty(M, device=cuda)
    dense._fused(Pt, Wp, bt, yt, 1.0 / T, None, G, loss, hits, wt)
    assert np.abs(loss.cpu().numpy() - w * loss64).max() < 1e-5 * w.max()
    assert np.abs(G.cpu().numpy() - w[:, None] * G64).max() < 1e-5 * w.max() / T + 1e-7
    srt = np.sort(logits64, axis=1)
    clear = (srt[:, -1] - srt[:, -2]) > 1e-4
    assert np.array_equal(hits.cpu().numpy()[clear], (w * hits64)[clear])
    loss_e = torch.empty(M, device=cuda)
    dense._fused(Pt, Wp, bt, yt, 1.0, None, None, loss_e, None, wt)  # evaluation form
    assert torch.equal(loss_e, loss)
    # all-ones weights: bitwise the unweighted kernel
    G1, l1 = empty_dense(M, N, cuda), torch.empty(M, device=cuda)
    G0, l0 = empty_dense(M, N, cuda), torch.empty(M, device=cuda)
    dense._fused(Pt, Wp, bt, yt, 1.0 / M, None, G1, l1, None, torch.ones(M, device=cuda))
    dense._fused(Pt, Wp, bt, yt, 1.0 / M, None, G0, l0, None)
    assert torch.equal(G1, G0) and torch.equal(l1, l0)
    # the row kernel on the logits: loss / accuracy over the weighted list and its gradient
    L = torch.from_numpy(logits64.astype(np.float32)).to(cuda).requires_grad_()
    lw, aw = dense.softmax_xent(L, yt, denom=int(T), row_weight=wt)
    lw.backward()
    L64 = L.detach().cpu().numpy().astype(np.float64)
    _P, lr64, hr64, Gr64 = O.softmax_xent_f64(L64, y, scale=1.0 / T)
    assert abs(float(lw) - (w * lr64).sum() / T) < 1e-5 * max(1.0, abs(float(lw)))
    assert np.abs(L.grad.cpu().numpy() - w[:, None] * Gr64).max() < 1e-5 * w.max() / T + 1e-7


BF16_OVERFLOW = 3.3961e38  # |x| from here on rounds to Inf in bf16 (bf16 max + half an ulp)


def _nonfinite_operands(M, K, N, seed):
    """A, B with +-Inf, NaN, values past bf16's largest finite (|x| >= 3.3961e38 rounds plane 0
    to Inf) and a row / column pair whose products overflow, each in its own rows / columns."""
    A, B = _rand((M, K), seed), _rand((K, N), seed + 1)
    A[3, 7] = np.inf
    A[11, 0] = -np.inf
    A[20, K - 1] = 3.4e38
    A[29, 5] = -3.3999e38
    B[9, 4] = np.inf
    B[K - 2, 13] = 3.4e38
    A[40, :] = 1e20                  # row 40 x column 50: every product 1e40 -> Inf in f32
    B[:, 50] = 1e20
    A[45, 2] = np.nan
    return A, B


@pytest.mark.parametrize("M,K,N", [(64, 100, 70), (300, 301, 133), (1000, 300, 930)])
def test_gemm_nt_bf16x6_nonfinite_has_f32_semantics(cuda, M, K, N):
    """gcg_spmm.h: a bf16x6 tile whose result is not finite is recomputed on the f32 MFMA in the
    f32 kernel's k order. So an infinite operand gives +-Inf (not the planes' Inf - Inf = NaN),
    an operand above bf16's largest finite value is not lost to a NaN, an overflow gives Inf,
    NaN stays NaN: the rows / columns of such operands are bitwise the f32 kernel's, in every
    bf16x6 form (tiles 0..8 with the plane workspace, and the in-loop split); every non-finite
    output equals the f32 one; finite outputs within the float64 bar."""
    A, B = _nonfinite_operands(M, K, N, 70)
    bias = _rand((N,), 72)
    At, Bt = torch.from_numpy(A).to(cuda), _padded(B, cuda, transpose=True)
    bt = torch.from_numpy(bias).to(cuda)
    ref = dense.gemm_nt(At, Bt, bias=bt, math="f32").cpu().numpy()
    assert np.isinf(ref).any() and np.isnan(ref).any()
    special = lambda X: ~np.isfinite(X) | (np.abs(X) >= BF16_OVERFLOW)  # noqa: E731
    bad_rows = np.unique(np.nonzero(special(A))[0])
    bad_cols = np.unique(np.nonzero(special(B))[1])
    with np.errstate(all="ignore"):
        C64 = A.astype(np.float64) @ B.astype(np.float64) + bias
        bound = 2e-6 * (np.abs(A).astype(np.float64) @ np.abs(B).astype(np.float64)
                        + np.abs(bias)) + 1e-30
    fin = np.isfinite(ref)
    fin[bad_rows] = False
    fin[:, bad_cols] = False
    forms = [("bf16x6_inloop", 0)] + [("bf16x6", t) for t in range(9)]
    for math, tile in forms:
        C = dense.gemm_nt(At, Bt, bias=bt, math=math, tile=tile).cpu().numpy()
        assert np.array_equal(np.isnan(C), np.isnan(ref)), (math, tile)
        inf = np.isinf(ref)
        assert np.array_equal(C[inf], ref[inf]), (math, tile)  # the sign of every Inf
        assert np.array_equal(C[bad_rows], ref[bad_rows], equal_nan=True), (math, tile)
        assert np.array_equal(C[:, bad_cols], ref[:, bad_cols], equal_nan=True), (math, tile)
        assert (np.abs(C[fin] - C64[fin]) <= bound[fin]).all(), (math, tile)


@pytest.mark.parametrize("N", [129, 930])
def test_fused_bf16x6_nonfinite_has_f32_semantics(cuda, N):
    """The fused output layer on the bf16 matrix cores against the f32 MFMA one, with an
    infinite activation, a NaN, one past bf16's largest finite value (whose products all
    overflow to -Inf) and one product that overflows to +Inf: the same non-finite losses and
    gradient entries (NaN / Inf pattern) as the f32 kernel, every other row within f32
    rounding. (Rows whose logits are finite but ~1e19 are avoided: exp(v - max) of such rows
    is decided by the last rounding bit in either arithmetic.)"""
    M, K = 70, 40
    P, W = _rand((M, K), 81, 0.3), _rand((K, N), 82, 0.3)
    b = _rand((N,), 83)
    P[3, 5] = np.inf
    P[17, 9] = np.nan
    P[10, 1] = -3.4e38
    W[1, :] = 2.0        # row 10: every product -6.8e38 -> -Inf
    P[:, 2] = 0.0
    P[33, 2] = 1e20
    W[2, 7] = 1e20       # row 33 x column 7: 1e40 -> +Inf
    y = np.random.default_rng(84).integers(0, N, M).astype(np.int32)
    Pt, Wt, bt = (torch.from_numpy(v).to(cuda) for v in (P, W, b))
    yt = torch.from_numpy(y).to(cuda)
    Wp = dense.Projection().fwd.get(Wt, False)
    res = {}
    for math in ("f32", "bf16x6"):
        G = empty_dense(M, N, cuda)
        loss, hits = torch.empty(M, device=cuda), torch.empty(M, device=cuda)
        dense._fused(Pt, Wp, bt, yt, 1.0 / M, None, G, loss, hits, math=math)
        res[math] = (G.cpu().numpy(), loss.cpu().numpy(), hits.cpu().numpy())
    (Gf, lf, hf), (Gb, lb, hb) = res["f32"], res["bf16x6"]
    special = [3, 10, 17, 33]
    assert not np.isfinite(lf[special]).any()
    assert np.array_equal(np.isnan(lb), np.isnan(lf)) and np.array_equal(np.isinf(lb), np.isinf(lf))
    assert np.array_equal(np.isnan(Gb), np.isnan(Gf)) and np.array_equal(np.isinf(Gb), np.isinf(Gf))
    fin = np.isfinite(lf)
    assert fin.sum() == M - len(special)
    assert np.abs(lb[fin] - lf[fin]).max() < 1e-5
    assert np.abs(Gb[fin] - Gf[fin]).max() < 1e-6


@pytest.mark.parametrize("R,M,N", [(1000, 300, 930), (4097, 300, 256), (77, 64, 300), (33, 5, 7),
                                   (513, 256, 300), (20000, 300, 930), (64, 301, 129)])
def test_gemm_tn_bf16x6_vs_float64(cuda, R, M, N):
    """gcg_gemm_tn math GCG_MATH_BF16X6 (gemm_tn6_partial_kernel): the split-K weight gradient
    on the bf16 matrix cores -- error against float64 at most 1.25 x the f32 kernel's (and below
    2^-20 of sum |a||b|), ragged R / M / N (partial 32-row chunks inside a split: rows past a
    split must read 0, they belong to the next), deterministic."""
    rng = np.random.default_rng(R + M + N)
    A = (rng.choice([-1.0, 1.0], (R, M)) * 10.0 ** rng.uniform(-2, 2, (R, M))).astype(np.float32)
    B = (rng.choice([-1.0, 1.0], (R, N)) * 10.0 ** rng.uniform(-2, 2, (R, N))).astype(np.float32)
    At, Bt = torch.from_numpy(A).to(cuda), torch.from_numpy(B).to(cuda)
    C64 = A.astype(np.float64).T @ B.astype(np.float64)
    scale = np.abs(A).astype(np.float64).T @ np.abs(B).astype(np.float64) + 1e-30
    rel = {}
    for math in ("f32", "bf16x6"):
        C = dense.gemm_tn(At, Bt, math=math).cpu().numpy()
        assert np.array_equal(C, dense.gemm_tn(At, Bt, math=math).cpu().numpy())  # deterministic
        rel[math] = float((np.abs(C.astype(np.float64) - C64) / scale).max())
    assert rel["bf16x6"] <= 1.25 * rel["f32"] + 2.0 ** -24 and rel["bf16x6"] < 2.0 ** -20, rel


def test_gemm_tn_bf16x6_nonfinite_has_f32_semantics(cuda):
    """A tile of the bf16x6 TN kernel whose sums are not finite is recomputed with f32 products:
    Inf propagates with its sign, Inf * 0 and NaN give NaN -- the f32 kernel's NaN / Inf pattern;
    every other element within the float64 bar."""
    R, M, N = 300, 70, 90
    A, B = _rand((R, M), 91), _rand((R, N), 92)
    A[5, 3] = np.inf
    B[7, 11] = np.nan
    A[9, 40] = 3.39e38 * 1.002  # above bf16's largest finite value
    At, Bt = torch.from_numpy(A).to(cuda), torch.from_numpy(B).to(cuda)
    ref = dense.gemm_tn(At, Bt, math="f32").cpu().numpy()
    C = dense.gemm_tn(At, Bt, math="bf16x6").cpu().numpy()
    assert np.array_equal(np.isnan(C), np.isnan(ref)) and np.array_equal(np.isinf(C), np.isinf(ref))
    inf = np.isinf(ref)
    assert np.array_equal(C[inf], ref[inf])
    fin = np.isfinite(ref)
    with np.errstate(all="ignore"):
        C64 = A.astype(np.float64).T @ B.astype(np.float64)
        bound = 2e-6 * (np.abs(A).astype(np.float64).T @ np.abs(B).astype(np.float64)) + 1e-30
    ok = fin & np.isfinite(C64)
    assert (np.abs(C[ok] - C64[ok]) <= bound[ok]).all()
