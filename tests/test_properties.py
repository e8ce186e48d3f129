"""Hypothesis property tests: the host planner on CPU, SpMM parity on the GPU."""
import ctypes as C

import numpy as np
import pytest
import scipy.sparse as sps
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st


def _plan(indptr, task_nnz, ordered, rows=None):
    from graphconvgeo_amd import _native
    indptr = np.ascontiguousarray(indptr, dtype=np.int32)
    r = None if rows is None else np.ascontiguousarray(rows, dtype=np.int32)
    nt, nl, ns = C.c_int64(), C.c_int64(), C.c_int64()
    args = (indptr.size - 1, indptr.ctypes.data, None if r is None else r.ctypes.data,
            0 if r is None else r.size, task_nnz, ordered)
    _native.call("gcg_spmm_plan_host", *args, None, 0, C.byref(nt), None, 0, C.byref(nl), C.byref(ns))
    tasks = np.zeros((max(nt.value, 1), 4), np.int32)
    longs = np.zeros((max(nl.value, 1), 4), np.int32)
    _native.call("gcg_spmm_plan_host", *args, tasks.ctypes.data, nt.value, C.byref(nt),
                 longs.ctypes.data, nl.value, C.byref(nl), C.byref(ns))
    return tasks[: nt.value], longs[: nl.value], ns.value


@settings(max_examples=200, deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture])
@given(lens=st.lists(st.integers(0, 3000), min_size=0, max_size=200),
       task_nnz=st.sampled_from([0, 1, 7, 32, 256, 512, 4096]),
       ordered=st.booleans(), use_rows=st.booleans(), data=st.data())
def test_planner_partitions_work_exactly(native_lib, lens, task_nnz, ordered, use_rows, data):
    indptr = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    n = len(lens)
    rows = None
    if use_rows and n > 0:
        rows = np.array(data.draw(st.lists(st.integers(0, n - 1), min_size=0, max_size=300)), np.int32)
    n_out = n if rows is None else len(rows)
    tasks, longs, nslots = _plan(indptr, task_nnz, int(ordered), rows)
    if task_nnz > 0:
        W = task_nnz
    elif ordered:  # spmm.hip default_task_nnz: 128 for ordered plans, 256 at >= 256 per row
        cap = 256 if n > 0 and int(indptr[-1]) >= 256 * n else 128
        W = max(32, min(cap, int(indptr[-1]) // 32768))
    else:
        W = max(32, min(512, int(indptr[-1]) // 8192))
    covered = np.zeros(n_out, np.int64)
    seg = {}
    slots = set()
    slices = {}
    for a, b, c, d in tasks:
        if c == -4:  # column slice b of d of the row at position a (ordered): covered once
            slices.setdefault(a, []).append(b)
            covered[a] += b == 0
        elif d < 0:
            assert 0 <= a < b <= n_out
            covered[a:b] += 1
        else:
            r = a if rows is None else rows[a]
            assert indptr[r] <= b < c <= indptr[r + 1] and c - b <= W
            seg.setdefault(a, []).append((b, c))
            slots.add(d)
    for p, first, cnt, _ in longs:
        covered[p] += 1
        r = p if rows is None else rows[p]
        parts = sorted(seg[p])
        assert len(parts) == cnt and parts[0][0] == indptr[r] and parts[-1][1] == indptr[r + 1]
        assert all(parts[i][1] == parts[i + 1][0] for i in range(cnt - 1))  # contiguous, in order
    assert np.all(covered == 1)
    assert all(ks == [0, 1] for ks in slices.values())
    assert not slices or ordered
    assert slots == set(range(nslots))
    if ordered:
        assert nslots == 0


def _rand_csr(rng, n_rows, n_cols, max_len, dup, unsorted):
    lens = rng.integers(0, max_len + 1, n_rows)
    if n_rows:
        lens[rng.integers(0, n_rows)] = max_len * 20  # one long row
    indptr = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    nnz = int(indptr[-1])
    idx = rng.integers(0, n_cols, nnz).astype(np.int32)
    m = sps.csr_matrix((rng.standard_normal(nnz).astype(np.float32), idx, indptr), shape=(n_rows, n_cols))
    if not dup:
        m.sum_duplicates()
        if unsorted:
            for i in range(n_rows):
                s, e = m.indptr[i], m.indptr[i + 1]
                p = rng.permutation(e - s) + s
                m.indices[s:e] = m.indices[p]
                m.data[s:e] = m.data[p]
    return m


@pytest.mark.gpu
@settings(max_examples=40, deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture])
@given(n_rows=st.integers(0, 300), n_cols=st.integers(1, 300), K=st.integers(0, 700),
       max_len=st.integers(0, 40), dup=st.booleans(), unsorted=st.booleans(),
       mode=st.sampled_from(["rowwise", "ordered", "fast", "auto"]),
       bias=st.booleans(), relu=st.booleans(), seed=st.integers(0, 2**31 - 1))
def test_spmm_matches_oracle(cuda, n_rows, n_cols, K, max_len, dup, unsorted, mode, bias, relu, seed):
    import torch
    from graphconvgeo_amd import sparse as gs
    from oracle import gcn_oracle as O
    rng = np.random.default_rng(seed)
    H = _rand_csr(rng, n_rows, n_cols, max_len, dup, unsorted)
    Z = rng.standard_normal((n_cols, K)).astype(np.float32)
    b = rng.standard_normal(K).astype(np.float32) if bias else None
    A = gs.DeviceCSR.from_scipy(H, cuda)
    Y = gs.spmm(A, torch.from_numpy(Z).to(cuda), bias=None if b is None else torch.from_numpy(b).to(cuda),
                act="relu" if relu else None, mode=mode, task_nnz=64).cpu().numpy()
    ref = O.spmm_f32(H, Z, bias=b, act="relu" if relu else None)
    if mode in ("rowwise", "ordered"):
        assert np.array_equal(Y, ref)
    else:
        assert Y.shape == ref.shape
        if ref.size:
            tol = 1e-5 * max(1.0, float(np.abs(ref).max())) * 10
            assert np.abs(Y - ref).max() <= tol
