"""GPU SpGEMM (input convolution X_conv = H * X, main.py:530 / tensormain.py:114) vs scipy."""
import warnings

import functools

import numpy as np
import pytest
import scipy.sparse as sps
import torch

from graphconvgeo_amd import sparse as gs
from graphconvgeo_amd.graph import normalize_edges_device, normalized_values_f64
from graphconvgeo_amd.synth import powerlaw_edges, synthetic_features

pytestmark = pytest.mark.gpu


def canon(m):
    m = sps.csr_matrix(m)
    m.sort_indices()
    return m


def test_spgemm_f32_bitwise_vs_scipy(cuda):
    rng = np.random.default_rng(0)
    A = sps.random(700, 500, density=0.02, random_state=1, format="csr", dtype=np.float32)
    A.data = rng.standard_normal(A.nnz).astype(np.float32)
    B = sps.random(500, 300, density=0.05, random_state=2, format="csr", dtype=np.float32)
    B.data = rng.standard_normal(B.nnz).astype(np.float32)
    C = gs.spgemm(gs.DeviceCSR.from_scipy(A, cuda), gs.DeviceCSR.from_scipy(B, cuda)).to_scipy()
    ref = canon(A @ B)  # scipy float32 csr_matmat: zero sums dropped
    assert np.array_equal(C.indptr, ref.indptr)
    assert np.array_equal(C.indices, ref.indices)
    assert np.array_equal(C.data, ref.data)


def test_spgemm_exact_zero_sums_dropped(cuda):
    A = sps.csr_matrix(np.array([[1.0, 1.0], [0.0, 2.0]], np.float32))
    B = sps.csr_matrix(np.array([[1.0, -1.0], [-1.0, 1.0]], np.float32))
    C = gs.spgemm(gs.DeviceCSR.from_scipy(A, cuda), gs.DeviceCSR.from_scipy(B, cuda)).to_scipy()
    assert C.nnz == (A @ B).nnz == 2
    assert np.array_equal(C.toarray(), (A @ B).toarray())


def test_input_convolution_reference_semantics(cuda):
    """X_conv = (H64 * X32).tocsr().astype('float32') with H built as tensormain.py:170-180."""
    n, e, f = 9_475, 80_000, 2_000
    u, v = powerlaw_edges(n, e)
    Hd = normalize_edges_device(n, u, v, cuda)
    X = synthetic_features(n, f, nnz_per_row=32)
    H64 = sps.csr_matrix((normalized_values_f64(Hd).cpu().numpy(), Hd.indices.cpu().numpy(),
                          Hd.indptr.cpu().numpy()), shape=(n, n))
    Xd = gs.DeviceCSR.from_scipy(X, cuda)
    C = gs.spgemm(Hd, Xd, a_data64=normalized_values_f64(Hd)).to_scipy()
    ref = canon((H64 * X).tocsr().astype("float32"))
    assert np.array_equal(C.indptr, ref.indptr)
    assert np.array_equal(C.indices, ref.indices)
    assert np.array_equal(C.data, ref.data)
    # float64 values equal the literal reference expression's
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        adj = sps.csr_matrix((np.ones(2 * e), (np.r_[u, v], np.r_[v, u])), shape=(n, n))
        adj.setdiag(1)
    d = np.asarray(adj.sum(axis=1)).flatten()
    D = sps.spdiags(1.0 / np.sqrt(d), [0], n, n, format="csr")
    H_lit = D * adj * D  # unsorted float64 (tensormain.py:180 before astype)
    ref_lit = canon((H_lit * X).tocsr().astype("float32"))
    assert np.array_equal(ref_lit.indices, C.indices)
    # the literal product sums in H_lit's storage order: equal to float32 rounding
    assert np.allclose(ref_lit.data, C.data, rtol=2e-7, atol=0)


def test_spgemm_empty(cuda):
    A = sps.csr_matrix((5, 4), dtype=np.float32)
    B = sps.random(4, 3, density=0.5, random_state=0, format="csr", dtype=np.float32)
    C = gs.spgemm(gs.DeviceCSR.from_scipy(A, cuda), gs.DeviceCSR.from_scipy(B, cuda))
    assert C.nnz == 0 and C.to_scipy().shape == (5, 3)
    with pytest.raises(ValueError):
        gs.spgemm(gs.DeviceCSR.from_scipy(B, cuda), gs.DeviceCSR.from_scipy(B, cuda))


@pytest.mark.parametrize("chunk", [1, 37, 1000, 50_000])
def test_spgemm_row_chunks_bitwise(cuda, chunk):
    """Row-chunked expand-sort-reduce (products > int32 at Twitter-World scale): forcing tiny
    chunks -- single rows larger than a chunk, chunks of empty rows -- leaves C bitwise equal."""
    sg = functools.partial(gs.spgemm, paths=("expand_sort",), chunk_products=chunk)
    rng = np.random.default_rng(chunk)
    A = sps.random(900, 400, density=0.03, random_state=3, format="lil", dtype=np.float32)
    A[100:220, :] = 0          # a block of empty rows
    A[5, :] = 1.0              # one dense row (400 * ~15 products)
    A = sps.csr_matrix(A)
    A.data = rng.standard_normal(A.nnz).astype(np.float32)
    B = sps.random(400, 250, density=0.04, random_state=4, format="lil", dtype=np.float32)
    B[7:30, :] = 0             # rows of A pointing at empty rows of B
    B = sps.csr_matrix(B)
    B.data = rng.standard_normal(B.nnz).astype(np.float32)
    # exact cancellations: column 0 of C gets +x and -x from two rows of B
    B = sps.lil_matrix(B)
    B[1, 0], B[2, 0] = 1.0, -1.0
    B = sps.csr_matrix(B)
    A = sps.lil_matrix(A)
    A[600, 1], A[600, 2] = 2.0, 2.0
    A = sps.csr_matrix(A)
    C = sg(gs.DeviceCSR.from_scipy(A, cuda), gs.DeviceCSR.from_scipy(B, cuda)).to_scipy()
    ref = canon(A @ B)
    assert np.array_equal(C.indptr, ref.indptr)
    assert np.array_equal(C.indices, ref.indices)
    assert np.array_equal(C.data, ref.data)
    A64 = torch.as_tensor(A.data.astype(np.float64) * 1.0000001, device=cuda)
    C64 = sg(gs.DeviceCSR.from_scipy(A, cuda), gs.DeviceCSR.from_scipy(B, cuda), a_data64=A64).to_scipy()
    A64h = sps.csr_matrix((A64.cpu().numpy(), A.indices, A.indptr), shape=A.shape)
    ref64 = canon((A64h @ B.astype(np.float64)).astype(np.float32))
    assert np.array_equal(C64.indptr, ref64.indptr) and np.array_equal(C64.indices, ref64.indices)
    assert np.array_equal(C64.data, ref64.data)


@pytest.mark.parametrize("path", ["rows", "dense", "esc"])
@pytest.mark.parametrize("p", [300, 30_000, 60_000])
def test_spgemm_rows_kernel_shapes(cuda, path, p):
    """The row-wise kernels (small rows: LDS sort; large rows: dense LDS slabs) across their regimes: several column slabs
    (p > 25,600 f32 / 13,312 f64), rows with > 2,048 products (several staging windows) and
    > 1,024 nonzeros (several step blocks), B rows longer than a wave, empty rows of A and B,
    exact cancellations -- bitwise scipy, f32 and f64 accumulation, both SpGEMM paths."""
    sg = functools.partial(gs.spgemm, paths={"rows": (), "dense": ("dense_slabs",), "esc": ("expand_sort",)}[path])
    rng = np.random.default_rng(p)
    m, n = 400, 3000
    A = sps.random(m, n, density=0.004, random_state=5, format="lil", dtype=np.float32)
    A[3, :] = 1.0                         # 3,000 nonzeros: 3 step blocks
    A[10, :1500] = 1.0
    A[50:80, :] = 0                       # empty rows
    A = sps.csr_matrix(A)
    A.data = rng.standard_normal(A.nnz).astype(np.float32)
    nnz_row = rng.integers(0, 200, n)     # B rows of 0..199 entries (several lanes rounds)
    nnz_row[:40] = 0
    rows = np.repeat(np.arange(n), nnz_row)
    cols = np.concatenate([rng.choice(p, k, replace=False) for k in nnz_row])
    B = sps.csr_matrix((rng.standard_normal(rows.size).astype(np.float32), (rows, cols)), shape=(n, p))
    B.sort_indices()
    # cancellation: C[7, c] = x - x
    B = sps.lil_matrix(B)
    B[1000, p - 1], B[1001, p - 1] = 3.0, -3.0
    B = sps.csr_matrix(B)
    A = sps.lil_matrix(A)
    A[7, :] = 0
    A[7, 1000], A[7, 1001] = 0.5, 0.5
    A = sps.csr_matrix(A)
    Ad, Bd = gs.DeviceCSR.from_scipy(A, cuda), gs.DeviceCSR.from_scipy(B, cuda)
    C = sg(Ad, Bd).to_scipy()
    ref = canon(A @ B)
    assert C[7, p - 1] == 0 and ref[7, p - 1] == 0
    assert np.array_equal(C.indptr, ref.indptr)
    assert np.array_equal(C.indices, ref.indices)
    assert np.array_equal(C.data, ref.data)
    a64 = torch.as_tensor(A.data.astype(np.float64) / 3.0, device=cuda)
    C64 = sg(Ad, Bd, a_data64=a64).to_scipy()
    A64 = sps.csr_matrix((a64.cpu().numpy(), A.indices, A.indptr), shape=A.shape)
    ref64 = canon((A64 @ B.astype(np.float64)).astype(np.float32))
    assert np.array_equal(C64.indptr, ref64.indptr) and np.array_equal(C64.indices, ref64.indices)
    assert np.array_equal(C64.data, ref64.data)
    Cacc = sg(Ad, Bd, accumulate_f64=True).to_scipy()  # f32 A, float64 sums
    refacc = canon((A.astype(np.float64) @ B.astype(np.float64)).astype(np.float32))
    assert np.array_equal(Cacc.indices, refacc.indices) and np.array_equal(Cacc.data, refacc.data)


@pytest.mark.parametrize("compact", ["inplace", "tmp"])
def test_spgemm_compaction_forms(cuda, compact):
    """C rows are computed at their product offsets inside c_idx/c_val and compacted there (row
    ranges whose destinations precede their sources), or through an nnz(C) temporary when that
    would take too many launches. Rows that merge nothing (in place), rows that merge a little
    (short ranges, single rows overlapping themselves) and rows that merge a lot, mixed."""
    sg = functools.partial(gs.spgemm, paths=("compact_temporary",) if compact == "tmp" else ())
    rng = np.random.default_rng(11)
    n, p = 3000, 5000
    # rows of A: first 500 rows one step each (no merging: in place), then rows of 2 steps
    # sharing a few columns (small gaps), then dense rows sharing many columns
    rows, cols = [], []
    for i in range(n):
        k = 1 if i < 500 else (2 if i < 2000 else 40)
        rows += [i] * k
        cols += list(rng.choice(n, k, replace=False))
    A = sps.csr_matrix((rng.standard_normal(len(rows)).astype(np.float32), (rows, cols)), shape=(n, n))
    B = sps.random(n, p, density=0.01, random_state=6, format="csr", dtype=np.float32)
    B.data = rng.standard_normal(B.nnz).astype(np.float32)
    C = sg(gs.DeviceCSR.from_scipy(A, cuda), gs.DeviceCSR.from_scipy(B, cuda)).to_scipy()
    ref = canon(A @ B)
    assert ref.nnz < int(np.diff(B.indptr)[A.indices].sum())  # some rows merged
    assert np.array_equal(C.indptr, ref.indptr)
    assert np.array_equal(C.indices, ref.indices)
    assert np.array_equal(C.data, ref.data)
