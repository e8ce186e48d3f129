"""GPU parity of the HIP SpMM (S.dot, mlpconv.py:71,73,90) against the CPU oracle.

Bar: 'rowwise' and 'ordered' modes are bitwise equal to the oracle (= scipy float32
csr_matvecs); 'fast' mode is within 1e-5 absolute of the float64 product on
normalized-H inputs (BASELINE.json north_star tolerance) and bitwise on every row it
does not split.
"""
import numpy as np
import pytest
import scipy.sparse as sps
import torch

from graphconvgeo_amd import sparse as gs
from graphconvgeo_amd.synth import synthetic_graph, dense
from oracle import gcn_oracle as O

pytestmark = pytest.mark.gpu

TOL = 1e-5  # north_star: "outputs match the Theano/scipy CPU reference within 1e-5 fp32"


def rand_csr(n_rows, n_cols, density_rows, seed, long_rows=(), empty_frac=0.1, sort=True,
             dups=False):
    rng = np.random.default_rng(seed)
    lens = rng.poisson(density_rows, size=n_rows)
    lens[rng.random(n_rows) < empty_frac] = 0
    for r, L in long_rows:
        lens[r] = L
    indptr = np.zeros(n_rows + 1, dtype=np.int64)
    np.cumsum(lens, out=indptr[1:])
    nnz = int(indptr[-1])
    indices = rng.integers(0, n_cols, size=nnz).astype(np.int32)
    if not dups:
        m = sps.csr_matrix((np.ones(nnz), indices, indptr), shape=(n_rows, n_cols))
        m.sum_duplicates()
        indptr, indices = m.indptr, m.indices.astype(np.int32)
        nnz = indices.size
    data = (rng.random(nnz) * 0.2 - 0.05).astype(np.float32)
    m = sps.csr_matrix((data, indices, indptr.astype(np.int32)), shape=(n_rows, n_cols))
    if not sort:
        for i in range(n_rows):
            s, e = m.indptr[i], m.indptr[i + 1]
            p = rng.permutation(e - s) + s
            m.indices[s:e] = m.indices[p]
            m.data[s:e] = m.data[p]
        m.has_sorted_indices = False
    return m


def to_dev(x, dev):
    return torch.from_numpy(np.ascontiguousarray(x)).to(dev)


@pytest.mark.parametrize("K", [1, 3, 4, 8, 63, 64, 65, 129, 256, 300, 512, 513, 930, 1500])
@pytest.mark.parametrize("mode", ["rowwise", "ordered"])
def test_bitwise_vs_oracle(cuda, K, mode):
    H = rand_csr(700, 500, 12, seed=K, long_rows=[(5, 3000), (600, 1500)])
    Z = np.random.default_rng(K).standard_normal((500, K)).astype(np.float32)
    A = gs.DeviceCSR.from_scipy(H, cuda)
    Y = gs.spmm(A, to_dev(Z, cuda), mode=mode).cpu().numpy()
    ref = O.spmm_f32(H, Z)
    assert np.array_equal(Y, ref), np.abs(Y - ref).max()


@pytest.mark.parametrize("K", [1, 3, 63, 65, 129, 301, 513, 930])
@pytest.mark.parametrize("mode", ["rowwise", "ordered", "fast"])
def test_masked_tail_vec4_bitwise(cuda, K, mode):
    """K % 4 != 0 on rows padded to a multiple of 4 floats (empty_dense; C = 930 -> 960): dwordx4
    gathers with a masked last vector (spmm.hip TL = 1). Bitwise equal to the narrower gathers of
    the same Z on unpadded rows (row stride K: dwordx2 / dword vectors) and to the oracle, with
    bias + rectify + gate bytes, a row subset with duplicates, cooperative hub rows (ordered) and
    split rows (fast); Y's and the gate's padding columns are never written."""
    H = rand_csr(700, 900, 12, seed=K, long_rows=[(5, 4500), (600, 1500)])
    Z = np.random.default_rng(K).standard_normal((900, K)).astype(np.float32)
    b = np.random.default_rng(K + 1).standard_normal(K).astype(np.float32)
    rows = np.random.default_rng(6).integers(0, 700, size=300).astype(np.int32)
    rows[:4] = 5
    A = gs.DeviceCSR.from_scipy(H, cuda)
    Zd = gs.empty_dense(900, K, cuda).copy_(to_dev(Z, cuda))
    Zd.as_strided((900, Zd.stride(0)), (Zd.stride(0), 1))[:, K:] = float("nan")  # padding
    Zn = to_dev(Z, cuda).contiguous()  # row stride K: the narrow gathers
    assert Zd.stride(0) % 4 == 0 and (K % 4 == 0 or Zn.stride(0) % 4 != 0)
    bd = to_dev(b, cuda)
    outs = {}
    for name, Zx in (("vec4", Zd), ("narrow", Zn)):
        Y = gs.empty_dense(700, K, cuda)
        Yfull = Y.as_strided((700, Y.stride(0)), (Y.stride(0), 1))
        Yfull.fill_(7.0)
        gate = gs.empty_gate(700, K, cuda)
        gfull = gate.as_strided((700, gate.stride(0)), (gate.stride(0), 1))
        gfull.fill_(9)
        gs.spmm(A, Zx, bias=bd, act="relu", mode=mode, gate=gate, out=Y, task_nnz=256)
        Ys = gs.spmm(A, Zx, rows=gs.RowSelection(rows, cuda), mode=mode, task_nnz=256)
        assert torch.all(Yfull[:, K:] == 7.0) and torch.all(gfull[:, K:] == 9)
        outs[name] = (Y.cpu().numpy(), gate.cpu().numpy(), Ys.cpu().numpy())
    for a, c in zip(outs["vec4"], outs["narrow"]):
        assert np.array_equal(a, c)
    Y, gate, Ys = outs["vec4"]
    if mode == "fast":
        assert np.abs(Y - O.spmm_f32(H, Z, bias=b, act="relu")).max() <= 1e-5
    else:
        pre = O.spmm_f32(H, Z, bias=b)
        assert np.array_equal(Y, O.relu(pre)) and np.array_equal(Ys, O.spmm_f32(H, Z, rows=rows))
        assert np.array_equal(gate, (2 * (pre > 0) + (pre == 0)).astype(np.uint8))


@pytest.mark.parametrize("K", [1, 4, 65, 300, 930])
@pytest.mark.parametrize("task_nnz", [16, 64, 512])
def test_fast_mode_tolerance(cuda, K, task_nnz):
    H = rand_csr(900, 800, 20, seed=7 + K, long_rows=[(3, 5000), (4, 700), (899, 2049)])
    Z = np.random.default_rng(K).standard_normal((800, K)).astype(np.float32)
    A = gs.DeviceCSR.from_scipy(H, cuda)
    Y = gs.spmm(A, to_dev(Z, cuda), mode="fast", task_nnz=task_nnz).cpu().numpy()
    ref32 = O.spmm_f32(H, Z)
    ref64 = O.spmm_f64(H, Z)
    assert np.abs(Y - ref64).max() <= TOL + np.abs(ref32 - ref64).max()
    lens = np.diff(H.indptr)
    unsplit = lens <= task_nnz
    assert np.array_equal(Y[unsplit], ref32[unsplit])
    info = A.plan(None, False, task_nnz).info()
    assert info["n_long_rows"] == int((~unsplit).sum())


def test_normalized_graph_fast_within_1e5(cuda):
    H = synthetic_graph(20_000, 200_000)  # power-law, hubs split in fast mode
    Z = dense(20_000, 300)
    A = gs.DeviceCSR.from_scipy(H, cuda, symmetric=True)
    Y = gs.spmm(A, to_dev(Z, cuda), task_nnz=128).cpu().numpy()
    ref64 = O.spmm_f64(H, Z)
    assert np.abs(Y - ref64).max() <= TOL
    assert A.plan(None, False, 128).info()["n_long_rows"] > 0


@pytest.mark.parametrize("mode", ["rowwise", "ordered", "fast"])
def test_bias_relu_and_rows_subset(cuda, mode):
    H = rand_csr(400, 300, 9, seed=3, long_rows=[(17, 900)])
    K = 129
    Z = np.random.default_rng(1).standard_normal((300, K)).astype(np.float32)
    b = np.random.default_rng(2).standard_normal(K).astype(np.float32)
    rows = np.random.default_rng(4).integers(0, 400, size=250).astype(np.int32)
    rows[:5] = 17  # duplicates, the long row (train indices are drawn with replacement)
    A = gs.DeviceCSR.from_scipy(H, cuda)
    sel = gs.RowSelection(rows, cuda)
    Y = gs.spmm(A, to_dev(Z, cuda), bias=to_dev(b, cuda), act="relu", rows=sel, mode=mode,
                task_nnz=256).cpu().numpy()
    ref = O.spmm_f32(H, Z, bias=b, act="relu", rows=rows)
    if mode == "fast":
        assert np.abs(Y - ref).max() <= 1e-5
    else:
        assert np.array_equal(Y, ref)
    # plain cuda index tensor -> plan-less path
    Y2 = gs.spmm(A, to_dev(Z, cuda), bias=to_dev(b, cuda), act="relu",
                 rows=to_dev(rows, cuda)).cpu().numpy()
    assert np.array_equal(Y2, ref)


@pytest.mark.parametrize("K", [4, 16, 60, 64, 68, 96, 124, 128])
def test_narrow_rows_subwave_path(cuda, K):
    """Narrow rows: plan-less (rowwise) launches run 4 rows per wave at K <= 64 and 2 at K <= 96
    (spmm_rows_kernel<4, 1, 16, 4, SUB>, one lane group per row); the planned modes run one row
    per wave. Rowwise bitwise equal to ordered and to the oracle, with bias + rectify + gate
    bytes, a row subset with duplicates, empty rows and a cooperative hub row (ordered); fast
    (split rows) within 1e-5, bitwise on unsplit rows."""
    H = rand_csr(777, 600, 10, seed=11 + K, long_rows=[(9, 4100), (500, 700)], empty_frac=0.15)
    Z = np.random.default_rng(K).standard_normal((600, K)).astype(np.float32)
    b = np.random.default_rng(K + 1).standard_normal(K).astype(np.float32)
    rows = np.random.default_rng(5).integers(0, 777, size=401).astype(np.int32)
    rows[:3] = 9
    A = gs.DeviceCSR.from_scipy(H, cuda)
    Zd, bd = to_dev(Z, cuda), to_dev(b, cuda)
    outs = {}
    for mode in ("rowwise", "ordered", "fast"):
        gate = gs.empty_gate(H.shape[0], K, cuda)
        Y = gs.spmm(A, Zd, bias=bd, act="relu", mode=mode, gate=gate, task_nnz=256)
        Ys = gs.spmm(A, Zd, rows=gs.RowSelection(rows, cuda), mode=mode, task_nnz=256)
        outs[mode] = (Y.cpu().numpy(), gate.cpu().numpy(), Ys.cpu().numpy())
    for a, c in zip(outs["rowwise"], outs["ordered"]):
        assert np.array_equal(a, c)
    Y, gate, Ys = outs["ordered"]
    ref = O.spmm_f32(H, Z, bias=b, act="relu")
    pre = O.spmm_f32(H, Z, bias=b)
    assert np.array_equal(Y, ref) and np.array_equal(Ys, O.spmm_f32(H, Z, rows=rows))
    want = np.where(pre > 0, 2, np.where(pre == 0, 1, 0)).astype(np.uint8)
    assert np.array_equal(gate, want)
    Yf = outs["fast"][0]
    assert np.abs(Yf - ref).max() <= 1e-5
    unsplit = np.diff(H.indptr) <= 256
    assert np.array_equal(Yf[unsplit], ref[unsplit])


@pytest.mark.parametrize("mode", ["ordered", "fast"])
@pytest.mark.parametrize("K", [128, 256, 300, 512, 1500])
def test_gather_hint_is_cache_policy_only(cuda, mode, K, monkeypatch):
    """The gather hint (cold columns' rows gathered non-temporally, DeviceCSR.gather_hint ->
    gcg_spmm_csr_f32_planned_hint) changes the loads' cache policy only: bitwise the hint-less
    result and the oracle, with cooperative hub rows (ordered), split rows (fast), a row
    subset, bias + rectify + gate. Thresholds lowered so a test-sized graph takes the hint."""
    monkeypatch.setattr(gs, "GATHER_HINT", True)
    monkeypatch.setattr(gs, "GATHER_HINT_MIN_TABLE", 0)
    monkeypatch.setattr(gs, "GATHER_HINT_HOT_BYTES", 4 << 20)  # 2k-3.4k hot rows: 48-59 % of nnz
    H = synthetic_graph(20_000, 200_000)  # power-law: hub columns
    Z = dense(20_000, K)
    b = np.random.default_rng(K).standard_normal(K).astype(np.float32)
    rows = np.random.default_rng(3).integers(0, 20_000, size=5000).astype(np.int32)
    A = gs.DeviceCSR.from_scipy(H, cuda, symmetric=True)
    hint = A.gather_hint(4 * min(gs.row_stride(K), 512))
    assert hint is not None and int((hint < 0).sum()) > 0
    assert torch.equal(hint & 0x7FFFFFFF, A.indices)
    Zd = gs.empty_dense(20_000, K, cuda).copy_(to_dev(Z, cuda))
    outs = {}
    for off in ("0", "1"):
        monkeypatch.setattr(gs, "GATHER_HINT", off == "0")  # "1": the hint-less launch
        gate = gs.empty_gate(20_000, K, cuda)
        Y = gs.spmm(A, Zd, bias=to_dev(b, cuda), act="relu", mode=mode, gate=gate, task_nnz=256)
        Ys = gs.spmm(A, Zd, rows=gs.RowSelection(rows, cuda), mode=mode, task_nnz=256)
        outs[off] = (Y.cpu().numpy(), gate.cpu().numpy(), Ys.cpu().numpy())
    for a, c in zip(outs["0"], outs["1"]):
        assert np.array_equal(a, c)
    if mode == "ordered":
        assert np.array_equal(outs["0"][0], O.spmm_f32(H, Z, bias=b, act="relu"))
        assert np.array_equal(outs["0"][2], O.spmm_f32(H, Z, rows=rows))


def test_gather_hint_first_call_inside_capture(cuda, monkeypatch):
    """A hint first needed inside a HIP-graph capture cannot be built there (its build syncs):
    the captured launch runs without it (default cache policy, same result) and nothing is
    cached; the next eager call builds it."""
    monkeypatch.setattr(gs, "GATHER_HINT", True)
    monkeypatch.setattr(gs, "GATHER_HINT_MIN_TABLE", 0)
    monkeypatch.setattr(gs, "GATHER_HINT_HOT_BYTES", 4 << 20)
    H = synthetic_graph(20_000, 200_000)
    A = gs.DeviceCSR.from_scipy(H, cuda, symmetric=True)
    gs.spmm(A, gs.empty_dense(20_000, 16, cuda).normal_(), mode="ordered")  # plan (outside)
    Z = gs.empty_dense(20_000, 300, cuda).copy_(to_dev(dense(20_000, 300), cuda))
    out = gs.empty_dense(20_000, 300, cuda)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        gs.spmm(A, Z, out=out, mode="ordered")
    assert 4 * 2**20 // 1216 not in A.__dict__.get("_gather_hints", {})  # not built in the capture
    g.replay()
    torch.cuda.synchronize()
    eager = gs.spmm(A, Z, mode="ordered")  # builds and uses the hint
    assert A.gather_hint(1216) is not None and torch.equal(out, eager)


def test_gather_hint_off_where_it_does_not_pay(cuda, monkeypatch):
    """No hint on a small operand (the Infinity Cache holds it) or a graph without hub columns."""
    monkeypatch.setattr(gs, "GATHER_HINT", True)
    A = gs.DeviceCSR.from_scipy(synthetic_graph(20_000, 200_000), cuda, symmetric=True)
    assert A.gather_hint(1216) is None  # 24 MB operand < GATHER_HINT_MIN_TABLE
    U = gs.DeviceCSR.from_scipy(synthetic_graph(20_000, 200_000, kind="uniform"), cuda,
                                symmetric=True)
    old = gs.GATHER_HINT_MIN_TABLE, gs.GATHER_HINT_HOT_BYTES, gs.GATHER_HINT
    try:
        gs.GATHER_HINT_MIN_TABLE, gs.GATHER_HINT_HOT_BYTES, gs.GATHER_HINT = 0, 1 << 20, True
        assert U.gather_hint(1216) is None  # the top 862 columns hold < 25 % of the nonzeros
        assert A.gather_hint(1216) is not None  # ... the power-law graph's do
    finally:
        gs.GATHER_HINT_MIN_TABLE, gs.GATHER_HINT_HOT_BYTES, gs.GATHER_HINT = old


def test_unsorted_and_duplicate_entries(cuda):
    H = rand_csr(300, 300, 15, seed=9, sort=False, dups=True)
    assert not H.has_canonical_format
    Z = np.random.default_rng(5).standard_normal((300, 64)).astype(np.float32)
    A = gs.DeviceCSR.from_scipy(H, cuda)
    for mode in ("rowwise", "ordered"):
        Y = gs.spmm(A, to_dev(Z, cuda), mode=mode).cpu().numpy()
        assert np.array_equal(Y, O.spmm_f32(H, Z))
        assert np.array_equal(Y, (H @ Z).astype(np.float32))  # scipy itself


def test_strided_operands(cuda):
    H = rand_csr(256, 200, 10, seed=11)
    Zbig = np.random.default_rng(6).standard_normal((200, 310)).astype(np.float32)
    Zt = to_dev(Zbig, cuda)[:, 5:305]  # ldz = 310, misaligned start -> scalar path
    A = gs.DeviceCSR.from_scipy(H, cuda)
    Y = gs.spmm(A, Zt).cpu().numpy()
    assert np.array_equal(Y, O.spmm_f32(H, Zbig[:, 5:305]))
    out = torch.full((256, 400), 7.0, device=cuda)
    gs.spmm(A, Zt, out=out[:, :300])
    assert torch.all(out[:, 300:] == 7.0)
    assert np.array_equal(out[:, :300].cpu().numpy(), O.spmm_f32(H, Zbig[:, 5:305]))


def test_edge_cases(cuda):
    # all rows empty (nnz = 0): output = act(bias)
    H = sps.csr_matrix((50, 40), dtype=np.float32)
    A = gs.DeviceCSR.from_scipy(H, cuda)
    b = torch.linspace(-1, 1, 12, device=cuda)
    Y = gs.spmm(A, torch.randn(40, 12, device=cuda), bias=b, act="relu")
    assert torch.equal(Y, torch.relu(b).expand(50, 12))
    # zero rows / zero width
    H0 = sps.csr_matrix((0, 10), dtype=np.float32)
    A0 = gs.DeviceCSR.from_scipy(H0, cuda)
    assert gs.spmm(A0, torch.randn(10, 5, device=cuda)).shape == (0, 5)
    A1 = gs.DeviceCSR.from_scipy(rand_csr(20, 10, 3, seed=1), cuda)
    assert gs.spmm(A1, torch.randn(10, 0, device=cuda)).shape == (20, 0)
    # one single huge row
    Hh = rand_csr(3, 5000, 0, seed=2, long_rows=[(1, 4000)], empty_frac=0)
    Z = np.random.default_rng(3).standard_normal((5000, 300)).astype(np.float32)
    Ah = gs.DeviceCSR.from_scipy(Hh, cuda)
    for mode in ("rowwise", "ordered"):
        assert np.array_equal(gs.spmm(Ah, to_dev(Z, cuda), mode=mode).cpu().numpy(), O.spmm_f32(Hh, Z))
    Yf = gs.spmm(Ah, to_dev(Z, cuda), mode="fast").cpu().numpy()
    assert np.abs(Yf - O.spmm_f64(Hh, Z)).max() < 1e-4


def test_errors(cuda):
    H = rand_csr(20, 10, 3, seed=1)
    A = gs.DeviceCSR.from_scipy(H, cuda)
    with pytest.raises(ValueError):
        gs.spmm(A, torch.randn(11, 4, device=cuda))
    with pytest.raises(TypeError):
        gs.spmm(A, torch.randn(10, 4, device=cuda, dtype=torch.float64))
    with pytest.raises(ValueError):
        gs.spmm(A, torch.randn(10, 4))  # CPU tensor: no fallback
    with pytest.raises(ValueError, match="must be sparse"):
        gs.spmm(np.zeros((3, 3)), torch.randn(3, 4, device=cuda))
    bad = sps.csr_matrix((np.ones(3, np.float32), np.array([0, 1, 99], np.int32),
                          np.array([0, 2, 3], np.int32)), shape=(2, 10), copy=False)
    with pytest.raises(ValueError, match="invalid CSR"):
        gs.DeviceCSR.from_scipy(bad, cuda)


def test_transpose_and_scatter_add(cuda):
    X = rand_csr(500, 120, 8, seed=21, long_rows=[(3, 100)])
    A = gs.DeviceCSR.from_scipy(X, cuda)
    T = A.transpose().to_scipy()
    ref = X.T.tocsr()  # scipy csr transpose: stable within a row
    assert np.array_equal(T.indptr, ref.indptr)
    assert np.array_equal(T.indices, ref.indices)
    assert np.array_equal(T.data, ref.data)
    # X^T . G (the dW1 gradient, mlpconv.py:71) bitwise = scipy on the transposed CSR
    G = np.random.default_rng(2).standard_normal((500, 300)).astype(np.float32)
    Y = gs.spmm(A.transpose(), to_dev(G, cuda), mode="ordered").cpu().numpy()
    assert np.array_equal(Y, O.spmm_f32(ref, G))
    # scatter-add with duplicate indices
    idx = np.random.default_rng(3).integers(0, 50, size=400).astype(np.int32)
    src = np.random.default_rng(4).standard_normal((400, 33)).astype(np.float32)
    base = np.random.default_rng(5).standard_normal((50, 33)).astype(np.float32)
    seg_ptr, pos = gs.index_csr(to_dev(idx, cuda), 50)
    out = to_dev(base.copy(), cuda)
    gs.scatter_add_rows(out, seg_ptr, pos, to_dev(src, cuda))
    assert np.array_equal(out.cpu().numpy(), O.scatter_add_f32(base.copy(), idx, src))


def test_geotext_scale_vs_oracle(cuda):
    """Config 2: GEOTEXT-scale graph, hidden 300, fp32 parity vs the CPU reference."""
    H = synthetic_graph(9_475, 80_000)
    Z = dense(9_475, 300)
    A = gs.DeviceCSR.from_scipy(H, cuda, symmetric=True)
    Zd = to_dev(Z, cuda)
    ref = O.spmm_f32(H, Z)
    assert np.array_equal(gs.spmm(A, Zd, mode="ordered").cpu().numpy(), ref)
    assert np.array_equal(gs.spmm(A, Zd, mode="rowwise").cpu().numpy(), ref)
    assert np.abs(gs.spmm(A, Zd, mode="fast").cpu().numpy() - O.spmm_f64(H, Z)).max() <= TOL


def test_row_partitioned_device_path_world1(cuda):
    """RowPartitionedCSR on the GPU (world = 1): gather buffer, column remap, HIP SpMM."""
    from graphconvgeo_amd.distributed import RowPartitionedCSR
    H = synthetic_graph(5_000, 40_000)
    Z = dense(5_000, 300)
    part = RowPartitionedCSR(H, 0, 1, cuda)
    Y = part.spmm(to_dev(Z, cuda), mode="ordered").cpu().numpy()
    assert np.array_equal(Y, O.spmm_f32(H, Z))
    # explicit 3-way bounds, each "rank" computed in turn on the one device (no collective)
    bounds = np.array([0, 1700, 3300, 5000])
    got = np.zeros_like(Y)
    for r in range(3):
        p = RowPartitionedCSR(H, r, 3, cuda, bounds=bounds)
        full = torch.zeros((3 * p.block_rows, 300), device=cuda)
        for q in range(3):
            full[q * p.block_rows: q * p.block_rows + bounds[q + 1] - bounds[q]] = \
                to_dev(Z[bounds[q]:bounds[q + 1]], cuda)
        got[bounds[r]:bounds[r + 1]] = gs.spmm(p.A, full, mode="ordered").cpu().numpy()
    assert np.array_equal(got, O.spmm_f32(H, Z))


@pytest.mark.parametrize("chunks", [1, 3, 4])
def test_pipelined_partition_bitwise(cuda, chunks):
    from graphconvgeo_amd.distributed import RowPartitionedCSR
    H = synthetic_graph(4_000, 30_000)
    Z = dense(4_000, 300)
    part = RowPartitionedCSR(H, 0, 1, cuda)
    Y = gs.empty_dense(4_000, 300, cuda)
    part.spmm_pipelined(to_dev(Z, cuda), Y, n_chunks=chunks, mode="ordered")
    assert np.array_equal(Y.cpu().numpy(), O.spmm_f32(H, Z))


def test_plan_released_during_graph_capture_is_deferred(cuda):
    """A plan whose owner dies while a HIP graph is being captured (a GC pass can run inside
    the capture) must not hipFree there: destruction is deferred to the next plan creation."""
    import gc
    import torch
    from graphconvgeo_amd import sparse as gs
    from graphconvgeo_amd.synth import synthetic_graph
    H = synthetic_graph(3000, 20000)
    A = gs.DeviceCSR.from_scipy(H, cuda, symmetric=True)
    doomed = gs.DeviceCSR.from_scipy(H, cuda, symmetric=True)
    Z = torch.randn((3000, 16), device=cuda)
    Y = gs.spmm(A, Z, mode="ordered")
    gs.spmm(doomed, Z, mode="ordered")  # doomed now owns a plan
    doomed._self = doomed  # reference cycle: only the cycle collector frees it
    del doomed
    g = torch.cuda.CUDAGraph()
    out = torch.empty_like(Y)
    with torch.cuda.graph(g):
        gs.spmm(A, Z, out=out, mode="ordered")
        gc.collect()  # the doomed operator and its plan die inside the capture
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(out, Y)
    gs.spmm(gs.DeviceCSR.from_scipy(H, cuda, symmetric=True), Z, mode="ordered")  # flushes
    assert not gs._RETIRED_PLANS


def test_rows_transpose_equals_scipy(cuda):
    """(H[idx])^T built on the device: same entries, same within-row order (target order) as
    scipy's stable `H[idx].T.tocsr()`; duplicated targets stay separate entries; the SpMM with
    it equals the scatter-then-H^T form within fp32 rounding."""
    import numpy as np
    import torch
    from graphconvgeo_amd import sparse as gs
    from graphconvgeo_amd.synth import synthetic_graph
    from oracle import gcn_oracle as O
    H = synthetic_graph(5000, 40000)
    idx = np.random.default_rng(4).integers(0, 5000, size=3000).astype(np.int32)
    A = gs.DeviceCSR.from_scipy(H, cuda, symmetric=True)
    rows = gs.RowSelection(idx, cuda)
    T = A.rows_transpose(rows)
    ref = H[idx].T.tocsr()
    assert T.shape == ref.shape
    assert np.array_equal(T.indptr.cpu().numpy(), ref.indptr)
    assert np.array_equal(T.indices.cpu().numpy(), ref.indices)
    assert np.array_equal(T.data.cpu().numpy(), ref.data)
    assert A.rows_transpose(gs.RowSelection(idx, cuda)) is T  # cached by content
    g = np.random.default_rng(5).standard_normal((3000, 24)).astype(np.float32)
    got = gs.spmm(T, torch.from_numpy(g).to(cuda), mode="ordered").cpu().numpy()
    assert np.array_equal(got, O.spmm_f32(ref, g))  # bitwise vs the oracle on the same CSR
    full = np.zeros((5000, 24), np.float32)
    O.scatter_add_f32(full, idx, g)
    assert np.abs(got - O.spmm_f32(H, full)).max() < 1e-5
    empty = A.rows_transpose(gs.RowSelection(np.zeros(0, np.int32), cuda))
    assert empty.shape == (5000, 0) and empty.nnz == 0


@pytest.mark.parametrize("K", [1, 3, 64, 65, 300, 513, 930])
@pytest.mark.parametrize("task_nnz", [32, 128, 512])
def test_ordered_cooperative_long_rows_bitwise(cuda, K, task_nnz):
    """'ordered' rows longer than 8 x task_nnz run on a whole workgroup (spmm.hip coop_row:
    the storage-order sum handed from wave to wave through LDS). Rows of every length around
    the batch size (WPB x U), a row subset repeating the long rows, bias + rectify + gate:
    bitwise the oracle."""
    lens = [(3, 5000), (10, 8 * task_nnz + 1), (11, 8 * task_nnz + 64 * 3 + 17), (12, 8 * task_nnz + 64),
            (13, 8 * task_nnz + 65), (14, 4097), (20, 12189), (21, 8 * task_nnz)]
    H = rand_csr(400, 30000, 10, seed=K + task_nnz, long_rows=lens, dups=True)  # exact lengths
    Z = np.random.default_rng(K).standard_normal((30000, K)).astype(np.float32)
    b = np.random.default_rng(K + 1).standard_normal(K).astype(np.float32)
    A = gs.DeviceCSR.from_scipy(H, cuda)
    info = A.plan(None, True, task_nnz).info()
    assert info["n_long_rows"] == int((np.diff(H.indptr) > 8 * task_nnz).sum()) >= 4
    Y = gs.spmm(A, to_dev(Z, cuda), mode="ordered", task_nnz=task_nnz).cpu().numpy()
    assert np.array_equal(Y, O.spmm_f32(H, Z))
    rows = np.array([20, 3, 3, 7, 14, 10, 20, 0, 11, 12, 13, 21], np.int32)
    gate = gs.empty_gate(rows.size, K, cuda)
    Yr = gs.spmm(A, to_dev(Z, cuda), bias=to_dev(b, cuda), act="relu", rows=gs.RowSelection(rows, cuda),
                 mode="ordered", task_nnz=task_nnz, gate=gate).cpu().numpy()
    pre = O.spmm_f32(H, Z, bias=b, rows=rows)
    assert np.array_equal(Yr, O.relu(pre))
    assert np.array_equal(gate.cpu().numpy(), (2 * (pre > 0) + (pre == 0)).astype(np.uint8))


def test_ordered_cooperative_world_scale_block(cuda):
    """A Twitter-World-like power-law block (hub rows of ~12k nonzeros) in 'ordered' mode:
    every hub row on the cooperative path, sampled rows bitwise the oracle, hub rows included."""
    H = synthetic_graph(200_000, 3_000_000)
    n = H.shape[0]
    Z = dense(n, 300)
    A = gs.DeviceCSR.from_scipy(H, cuda, symmetric=True)
    # 128-nnz tasks: rows over 1024 nonzeros (hub rows up to 0.01 N = 2000) go cooperative
    assert A.plan(None, True, 128).info()["n_long_rows"] > 0
    Y = gs.spmm(A, to_dev(Z, cuda), mode="ordered", task_nnz=128).cpu().numpy()
    lens = np.diff(H.indptr)
    hubs = np.argsort(lens)[-64:]
    sample = np.unique(np.concatenate([hubs, np.random.default_rng(0).choice(n, 2000)]))
    assert np.array_equal(Y[sample], O.spmm_f32(H, Z, rows=sample))


@pytest.mark.parametrize("K", [1, 3, 64, 257, 300, 301, 930, 1500, 8200])
@pytest.mark.parametrize("task_nnz", [32, 128])
def test_ordered_sliced_hub_rows_bitwise(cuda, K, task_nnz):
    """'ordered' rows longer than 8 x task_nnz run on whole workgroups; in a launch two 256-float
    chunks wide those also past 1/768 of the plan's nonzeros (here: all) are cut into two column
    slices on two CUs (spmm.hip coop_slice, round 5),
    each summing every nonzero of the row for its columns in storage order. Bitwise the oracle:
    hub rows of every length around the batch, a row subset repeating the hub rows, bias +
    rectify + gate, padded operands with a masked last vector (K = 257, 930: dwordx4 + tail),
    unpadded odd widths (K = 301: dword gathers, one slice runs the whole row), several column
    panels (K = 930, 1500, 8200), repeated launches and HIP-graph replays; ordered plan 2
    (unsliced) gives the same bits."""
    lens = [(3, 5000), (20, 12189), (21, 3001), (40, 16 * task_nnz), (41, 16 * task_nnz + 777),
            (10, 8 * task_nnz + 1), (11, 12 * task_nnz)]
    n_cols = 30000 if K <= 1500 else 3000
    H = rand_csr(400, n_cols, 10, seed=K + task_nnz, long_rows=lens, dups=True)
    Z = np.random.default_rng(K).standard_normal((n_cols, K)).astype(np.float32)
    b = np.random.default_rng(K + 1).standard_normal(K).astype(np.float32)
    A = gs.DeviceCSR.from_scipy(H, cuda)
    info = A.plan(None, True, task_nnz).info()
    rl = np.diff(H.indptr)
    n_hub = int((rl > 8 * task_nnz).sum())
    assert rl[rl > 8 * task_nnz].min() * 768 >= H.nnz  # every hub row past 1/768 of the work
    assert info["n_coop_rows"] == info["n_sliced_rows"] == info["n_long_rows"] == n_hub >= 6
    assert info["n_slices"] == 2
    assert A.plan(None, 2, task_nnz).info()["n_sliced_rows"] == 0
    if K in (257, 930):
        Zd = gs.empty_dense(n_cols, K, cuda)  # padded rows: dwordx4 with a masked last vector
        Zd.copy_(to_dev(Z, cuda))
        assert Zd.stride(0) % 4 == 0 and Zd.stride(0) > K
    else:
        Zd = to_dev(Z, cuda)
    ref = O.spmm_f32(H, Z)
    Y = gs.spmm(A, Zd, mode="ordered", task_nnz=task_nnz)
    assert np.array_equal(Y.cpu().numpy(), ref)
    Y2 = gs.spmm(A, Zd, mode="ordered", task_nnz=task_nnz)
    assert torch.equal(Y, Y2)
    try:
        gs.ORDERED_PLAN = 2
        assert torch.equal(gs.spmm(A, Zd, mode="ordered", task_nnz=task_nnz), Y)
    finally:
        gs.ORDERED_PLAN = 1
    rows = np.array([20, 3, 3, 7, 41, 40, 20, 0, 11, 21, 10, 20], np.int32)
    sel = gs.RowSelection(rows, cuda)
    assert A.plan(sel, True, task_nnz).info()["n_sliced_rows"] == 10
    gate = gs.empty_gate(rows.size, K, cuda)
    Yr = gs.spmm(A, Zd, bias=to_dev(b, cuda), act="relu", rows=sel, mode="ordered",
                 task_nnz=task_nnz, gate=gate).cpu().numpy()
    pre = O.spmm_f32(H, Z, bias=b, rows=rows)
    assert np.array_equal(Yr, O.relu(pre))
    assert np.array_equal(gate.cpu().numpy(), (2 * (pre > 0) + (pre == 0)).astype(np.uint8))
    if K in (300, 930):  # replayed HIP graph
        out = gs.empty_dense(400, K, cuda)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            gs.spmm(A, Zd, out=out, mode="ordered", task_nnz=task_nnz)
        for _ in range(3):
            out.zero_()
            g.replay()
            torch.cuda.synchronize()
            assert np.array_equal(out.cpu().numpy(), ref)
