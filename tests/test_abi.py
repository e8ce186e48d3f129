"""CPU tests of the C-ABI library: it loads, exports every symbol include/gcg_spmm.h
declares, and its host-only planner balances work (no GPU compute here)."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "gcg_spmm.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(gcg_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_expected_entry_points():
    names = declared_functions()
    for must in ("gcg_spmm_csr_f32", "gcg_spmm_csr_f32_planned", "gcg_spmm_plan_create",
                 "gcg_spmm_plan_destroy", "gcg_scatter_add_rows_f32", "gcg_csr_transpose_f32"):
        assert must in names


def test_library_exports_every_declared_symbol(native_lib):
    from graphconvgeo_amd import _build, _native
    for name in declared_functions():
        assert hasattr(native_lib, name), name
        assert name in _native.SIGNATURES, f"{name} has no ctypes signature"
    nm = subprocess.run(["nm", "-D", "--defined-only", _native.lib_path()], capture_output=True,
                        text=True, check=True).stdout
    exported = set(re.findall(r"\bT (gcg_[a-z0-9_]+)$", nm, flags=re.M))
    assert set(declared_functions()) <= exported
    assert _native.version() == "0.2.0"
    assert _native.load().gcg_source_hash().decode() == _build.source_hash()


def test_header_compiles_as_c():
    src = f'#include "{HEADER}"\nint main(void) {{ return GCG_OK; }}\n'
    res = subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-x", "c", "-", "-o", "/dev/null"],
                         input=src, capture_output=True, text=True)
    assert res.returncode == 0, res.stderr


def plan_host(indptr, task_nnz=512, ordered=0, rows=None):
    from graphconvgeo_amd import _native
    indptr = np.ascontiguousarray(indptr, dtype=np.int32)
    rows_a = None if rows is None else np.ascontiguousarray(rows, dtype=np.int32)
    n = indptr.size - 1
    nt, nl, ns = C.c_int64(), C.c_int64(), C.c_int64()
    args = (n, indptr.ctypes.data, None if rows_a is None else rows_a.ctypes.data,
            0 if rows_a is None else rows_a.size, task_nnz, ordered)
    _native.call("gcg_spmm_plan_host", *args, None, 0, C.byref(nt), None, 0, C.byref(nl), C.byref(ns))
    tasks = np.zeros((max(nt.value, 1), 4), np.int32)
    longs = np.zeros((max(nl.value, 1), 4), np.int32)
    _native.call("gcg_spmm_plan_host", *args, tasks.ctypes.data, nt.value, C.byref(nt),
                 longs.ctypes.data, nl.value, C.byref(nl), C.byref(ns))
    return tasks[: nt.value], longs[: nl.value], ns.value


@pytest.mark.parametrize("ordered", [0, 1])
def test_planner_covers_every_row_once(native_lib, ordered):
    rng = np.random.default_rng(0)
    lens = rng.zipf(1.8, size=5000).clip(0, 20000)
    lens[rng.random(5000) < 0.1] = 0
    indptr = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    tasks, longs, nslots = plan_host(indptr, task_nnz=256, ordered=ordered)
    covered = np.zeros(5000, np.int64)
    seg_nnz = np.zeros(5000, np.int64)
    slices = {}
    for a, b, c, d in tasks:
        if c == -4:  # column slice b of d of the row at position a (ordered)
            assert ordered and d == 2
            slices.setdefault(a, []).append(b)
            covered[a] += b == 0
        elif d < 0:
            covered[a:b] += 1
            nnz = indptr[b] - indptr[a]
            assert nnz <= 256 or b - a == 1  # a task over budget is a single (unsplit) row
        else:
            seg_nnz[a] += c - b
            assert indptr[a] <= b < c <= indptr[a + 1] and 0 <= d < nslots
            assert c - b <= 256
    for p, first, cnt, _ in longs:
        covered[p] += 1
        assert seg_nnz[p] == lens[p]
    assert np.all(covered == 1)
    for ks in slices.values():  # both column slices, adjacent
        assert ks == [0, 1]
    if ordered:
        assert len(longs) == 0 and nslots == 0
        # rows past 8 x task_nnz and 1/768 of the work: two column slices, longest first, leading
        sliced = sorted(slices, key=lambda a: -int(lens[a]))
        slice_min = max(8 * 256, int(lens.sum()) // 768)
        assert len(slices) == int(((lens > 8 * 256) & (lens >= slice_min)).sum()) > 0
        first = [t[0] for t in tasks if t[2] == -4][::2]
        assert first == sliced and all(t[2] == -4 for t in tasks[:2 * len(first)])
    else:
        assert len(longs) == int((lens > 256).sum())


def test_planner_row_subset_and_errors(native_lib):
    from graphconvgeo_amd import _native
    indptr = np.array([0, 2, 2, 700, 705], np.int32)
    tasks, longs, ns = plan_host(indptr, task_nnz=100, rows=[3, 1, 1, 0])
    assert all(t[3] < 0 for t in tasks) and len(longs) == 0
    tasks, longs, ns = plan_host(indptr, task_nnz=100, rows=[2, 1, 1])
    assert longs[:, 0].tolist() == [0] and ns == 7
    with pytest.raises(_native.NativeError, match="INVALID_ARG"):
        plan_host(indptr, rows=[9])
    with pytest.raises(_native.NativeError, match="BAD_CSR"):
        plan_host(np.array([0, 5, 3], np.int32))


def test_row_partition_balance():
    from graphconvgeo_amd.distributed import remap_columns, row_partition
    rng = np.random.default_rng(1)
    lens = rng.zipf(2.0, 10000).clip(1, 3000)
    indptr = np.concatenate([[0], np.cumsum(lens)])
    for P in (1, 2, 3, 8):
        b = row_partition(indptr, P)
        assert b[0] == 0 and b[-1] == 10000 and np.all(np.diff(b) >= 0)
        cost = np.diff(indptr[b] + 2 * b)
        assert cost.max() <= cost.sum() / P + lens.max() + 2
    b = np.array([0, 3, 7, 10])
    assert remap_columns(np.array([0, 2, 3, 6, 7, 9]), b, 4).tolist() == [0, 2, 4, 7, 8, 10]


def test_product_path_refuses_cpu_tensors(native_lib):
    import scipy.sparse as sps
    import torch
    from graphconvgeo_amd import sparse as gs
    with pytest.raises(ValueError, match="CUDA"):
        gs.DeviceCSR.from_scipy(sps.eye(3, format="csr", dtype=np.float32), "cpu")
    with pytest.raises(ValueError, match="must be sparse"):
        gs.DeviceCSR.from_scipy(np.eye(3), "cpu")


def test_abi_argument_validation_without_gpu(native_lib):
    """Entry points validate sizes/pointers before touching the device."""
    from graphconvgeo_amd import _native
    lib = native_lib
    # negative sizes, NULL outputs, bad activation, ld < K
    assert lib.gcg_spmm_csr_f32(-1, 1, 0, None, None, None, None, 1, 1, None, 1, None, 0, None, 0, None) == 1
    assert lib.gcg_spmm_csr_f32(2, 2, 0, None, None, None, None, 4, 4, None, 4, None, 0, None, 0, None) == 1
    assert lib.gcg_spmm_plan_create(None, 1, 1, 0, None, None, 0, 0, 0, None) == 1
    assert lib.gcg_spmm_plan_destroy(None) == 0
    assert lib.gcg_spmm_csr_f32_planned(None, None, None, None, None, 1, 1, None, 1, None, 0, None, 0, None) == 1
    assert lib.gcg_scatter_add_rows_f32(-1, None, None, None, 1, 1, None, 1, None) == 1
    assert lib.gcg_spgemm(1, 1, 1, 0, None, None, None, 0, 0, None, None, None, 0, 0, None, None, None, None, None) == 1
    assert lib.gcg_spgemm_products(-1, 0, None, None, 0, None, None, None) == 1
    msg = lib.gcg_last_error().decode()
    assert msg  # a readable message for the last failure on this thread
    with pytest.raises(_native.NativeError, match="INVALID_ARG"):
        _native.call("gcg_spmm_csr_f32", -1, 1, 0, None, None, None, None, 1, 1, None, 1, None, 0, None, 0, None)


def test_plain_c_consumer(native_lib, tmp_path):
    """tests/c/abi_consumer.c builds with gcc against include/gcg_spmm.h and links the .so."""
    from graphconvgeo_amd import _native
    lib = _native.lib_path()
    exe = tmp_path / "abi_consumer"
    src = os.path.join(ROOT, "tests", "c", "abi_consumer.c")
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), src,
                    lib, f"-Wl,-rpath,{os.path.dirname(lib)}", "-o", str(exe)], check=True)
    res = subprocess.run([str(exe)], capture_output=True, text=True)
    assert res.returncode == 0, (res.returncode, res.stdout, res.stderr)
    assert "abi ok" in res.stdout


def test_dense_abi_argument_validation_without_gpu(native_lib):
    """The MFMA dense entry points (csrc/dense.hip) reject bad shapes, layouts and missing
    outputs before any launch: sizes, 16-B alignment / ld % 4 of the dwordx4 operands,
    ldb >= round4(N), the fused kernel's 1024-class row limit, the row kernel's 4096."""
    import ctypes as C
    lib = native_lib
    a16, b16, c16 = C.c_void_p(0x10000), C.c_void_p(0x20000), C.c_void_p(0x30000)
    odd = C.c_void_p(0x10004)  # 4-B but not 16-B aligned
    st = {"ok": 0, "inval": 1, "mis": 2}
    gemm = lib.gcg_gemm_f32
    assert gemm(-1, 4, 4, a16, 4, b16, 4, None, 0, c16, 4, None) == st["inval"]
    assert gemm(4, 0, 4, a16, 4, b16, 4, None, 0, c16, 4, None) == st["inval"]
    assert gemm(4, 4, 4, None, 4, b16, 4, None, 0, c16, 4, None) == st["inval"]
    assert gemm(4, 4, 4, a16, 4, b16, 4, None, 7, c16, 4, None) == st["inval"]   # act
    assert gemm(4, 4, 8, a16, 4, b16, 4, None, 0, c16, 4, None) == st["inval"]   # lda < K
    assert gemm(4, 6, 4, a16, 4, b16, 6, None, 0, c16, 8, None) == st["inval"]   # ldb < round4(N)
    assert gemm(4, 4, 4, odd, 4, b16, 4, None, 0, c16, 4, None) == st["mis"]
    assert gemm(4, 4, 6, a16, 6, b16, 4, None, 0, c16, 4, None) == st["mis"]     # lda % 4
    assert gemm(0, 4, 4, a16, 4, b16, 4, None, 0, c16, 4, None) == st["ok"]      # M = 0: no-op
    fused = lib.gcg_project_softmax_xent_f32
    lab, loss = C.c_void_p(0x40000), C.c_void_p(0x50000)
    assert fused(4, 1025, 4, a16, 4, b16, 1028, None, lab, 1.0, None, c16, 1028, loss, None,
                 None) == st["inval"]
    assert fused(4, 8, 4, a16, 4, b16, 8, None, lab, 1.0, None, c16, 8, None, None,
                 None) == st["inval"]                                           # no loss_rows
    assert fused(0, 8, 4, a16, 4, b16, 8, None, lab, 1.0, None, None, 0, loss, None,
                 None) == st["ok"]                                              # eval form, M = 0
    rows = lib.gcg_softmax_xent_f32
    assert rows(4, 4097, a16, 4100, lab, 1.0, None, c16, 4100, loss, None, None) == st["inval"]
    assert rows(4, 8, a16, 8, None, 1.0, None, None, 8, None, None, None) == st["inval"]
    assert rows(4, 8, a16, 4, lab, 1.0, None, None, 8, loss, None, None) == st["inval"]  # ldl < N
    assert "gcg_softmax_xent_f32" in lib.gcg_last_error().decode()


def test_gemm_tn_abi_without_gpu(native_lib):
    """Split-K weight-gradient GEMM: workspace sizing and argument checks run on the host."""
    import ctypes as C
    lib = native_lib
    nb = C.c_size_t()
    assert lib.gcg_gemm_tn_f32_workspace_bytes(840_000, 300, 930, C.byref(nb)) == 0
    # partials: splits x round64(M) x round192(N) floats (per-wave 64 x 192 tiles), ~2 waves
    # per SIMD over the launch
    assert nb.value % (4 * 320 * 960) == 0 and 40 <= nb.value // (4 * 320 * 960) <= 2048
    assert lib.gcg_gemm_tn_f32_workspace_bytes(0, 3, 5, C.byref(nb)) == 0 and nb.value == 0
    assert lib.gcg_gemm_tn_f32_workspace_bytes(-1, 3, 5, C.byref(nb)) == 1
    a16, b16, c16 = C.c_void_p(0x10000), C.c_void_p(0x20000), C.c_void_p(0x30000)
    tn = lib.gcg_gemm_tn_f32
    assert tn(8, 3, 5, a16, 4, b16, 8, None, c16, 5, None, 0, None) == 6      # no workspace
    assert tn(8, 3, 5, a16, 3, b16, 8, None, c16, 5, None, 0, None) == 1      # lda < round4(M)
    assert tn(8, 3, 5, C.c_void_p(0x10008), 4, b16, 8, None, c16, 5, None, 0, None) == 2
    assert tn(8, 3, 5, a16, 4, b16, 8, None, c16, 4, None, 0, None) == 1      # ldc < N


def test_relu_backward_abi_without_gpu(native_lib):
    """Fused rectify backward + bias gradient: workspace sizing and host-side checks."""
    import ctypes as C
    lib = native_lib
    nb = C.c_size_t()
    assert lib.gcg_relu_backward_f32_workspace_bytes(840_000, 300, C.byref(nb)) == 0
    assert nb.value == 4 * 300 * 1020  # at most 1024 partial rows (here 824 rows each) ...
    assert lib.gcg_relu_backward_f32_workspace_bytes(5000, 300, C.byref(nb)) == 0
    assert nb.value == 4 * 300 * 10     # ... of at least 512 rows each
    assert lib.gcg_relu_backward_f32_workspace_bytes(-1, 3, C.byref(nb)) == 1
    a16, b16, c16, w16 = (C.c_void_p(x) for x in (0x10000, 0x20000, 0x30000, 0x40000))
    rb = lib.gcg_relu_backward_f32
    assert rb(8, 1025, a16, 1028, b16, 1028, c16, 1028, None, w16, 1 << 20, None) == 1  # K cap
    assert rb(8, 4, None, 4, b16, 4, c16, 4, None, w16, 1 << 20, None) == 1            # null gY
    assert rb(8, 4, a16, 3, b16, 4, c16, 4, None, w16, 1 << 20, None) == 1             # ld < K
    assert rb(8, 4, C.c_void_p(0x10002), 4, b16, 4, c16, 4, None, w16, 1 << 20, None) == 2
    assert rb(8, 4, a16, 4, b16, 4, c16, 4, None, None, 0, None) == 6                  # workspace
    assert rb(8, 4, a16, 4, b16, 4, c16, 4, None, w16, 4, None) == 6                   # too small
    # K > 256 needs the dwordx4 path (16-B rows)
    assert rb(8, 300, a16, 301, b16, 304, c16, 304, None, w16, 1 << 20, None) == 2
    assert rb(0, 4, None, 4, None, 4, None, 4, None, None, 0, None) == 0               # empty


def test_column_sum_abi_without_gpu(native_lib):
    import ctypes as C
    cs = native_lib.gcg_column_sum_f32
    a16, o16, w16 = (C.c_void_p(x) for x in (0x10000, 0x20000, 0x40000))
    assert cs(8, 4, a16, 4, None, w16, 1 << 20, None) == 1           # null out
    assert cs(8, 4, a16, 3, o16, w16, 1 << 20, None) == 1            # ld < K
    assert cs(8, 1025, a16, 1028, o16, w16, 1 << 22, None) == 1      # K cap
    assert cs(8, 4, a16, 4, o16, None, 0, None) == 6                 # workspace
    assert cs(8, 300, a16, 301, o16, w16, 1 << 20, None) == 2        # wide needs 16-B rows
