"""HBM-resident CSR operators and the SpMM entry point (host mirror of `S.dot`).

`DeviceCSR` holds a scipy-layout CSR (indptr/indices int32, data float32) in HBM.
The reference keeps H as one host scipy matrix shared by both layers
(`H=l_hid1.H`, mlpconv.py:214); here it is uploaded once and every layer, epoch
and width K reuses the same device buffers and launch plans.

`spmm(A, Z, ...)` is `theano.sparse.dot(A, Z)` (mlpconv.py:71,73,90) with the
layer epilogue fused (bias, rectify, target-row subset). It always runs the HIP
kernels in libgcg_spmm.so; there is no CPU path.
"""
from __future__ import annotations

import ctypes as C
import hashlib
import itertools
import math
import os
import weakref
from typing import Optional, Union

import numpy as np
import scipy.sparse as sps
import torch

from . import _native
from ._native import GCG_ACT_NONE, GCG_ACT_RELU, call

ACTS = {None: GCG_ACT_NONE, "none": GCG_ACT_NONE, "linear": GCG_ACT_NONE,
        "relu": GCG_ACT_RELU, "rectify": GCG_ACT_RELU}

MODES = ("auto", "fast", "ordered", "rowwise")

# 'auto' runs the bitwise 'ordered' plan unless one row is long enough to outlast the
# whole launch (then rows are split, 'fast'). Round 2 set the limit at nnz/2048 (long rows then
# ran on one wave); since the ordered plan runs long rows on whole workgroups (round 3) and
# cuts hub rows into column slices (round 5), a row streams at ~19 GB/s per CU against ~6.5
# TB/s for the launch, i.e. it outlasts the launch only beyond ~nnz/340 (nnz/215 sliced).
# Round 5: nnz/512. The W1 gradient's tail gather (CSR(X^T) without the dense head, 43.5M
# nonzeros, longest row 43,164 = nnz/1008) ran 'fast' at 8.28 ms and runs 'ordered' -- bitwise
# -- at 7.82-7.89 ms (tools/exp_xt_tail.py, profiles/r05/xt_tail_modes.jsonl); Twitter-World
# H (12,189 of 41.4M) is ordered either way.
AUTO_SPLIT_RATIO = 512
# DeviceCSR.tmatmul moves the dense Zipf-head columns to the MFMA GEMM when CSR(X^T)'s longest
# row exceeds nnz / TMATMUL_SPLIT_RATIO (the round-2 rule, kept for that decision)
TMATMUL_SPLIT_RATIO = 2048
# ... and the plan-less 'rowwise' form (also bitwise) when no row is a hub: longest row at most
# AUTO_ROWWISE_SKEW x the mean, on a graph large enough to fill the chip with one wave per row.
# Measured on the Twitter-World uniform-degree graph (max 2.2x the mean), K = 300: 9.43 vs
# 9.63 ms for the 512-nnz task plan; on the power-law graph rowwise is 18 % slower (hub rows).
AUTO_ROWWISE_SKEW = 4
AUTO_ROWWISE_MIN_ROWS = 65536


def auto_mode(n_rows: int, nnz: int, longest: int) -> str:
    """The mode 'auto' picks for a CSR of n_rows rows, nnz nonzeros and longest row `longest`."""
    nnz = max(int(nnz), 1)
    if longest * AUTO_SPLIT_RATIO > nnz:
        return "fast"
    if n_rows >= AUTO_ROWWISE_MIN_ROWS and longest * n_rows <= AUTO_ROWWISE_SKEW * nnz:
        return "rowwise"
    return "ordered"


def resolve_auto(A) -> str:
    """The mode 'auto' runs on A: 'fast', 'rowwise' or 'ordered' (see above)."""
    return auto_mode(A.n_rows, A.nnz, A.max_row_nnz())

# DeviceCSR.tmatmul: columns at least this dense (fraction of rows) leave the CSR gather for
# the dense MFMA GEMM -- break-even is ~1.5-2 % (a gathered nonzero ~190 ps, a dense element
# ~3-9 ps at Twitter-World, round-1 measurements; the head size re-checked in round 2 with
# tools/exp_hybrid_cols.py, profiles/HISTORY.md §7); at most HYBRID_MAX_COLS
# of them (the GEMM's cost grows faster than the gather it saves beyond), and only
# for matrices of at least HYBRID_MIN_ROWS rows (below that everything is cache-resident).
HYBRID_MIN_DENSITY = 0.02
HYBRID_MAX_COLS = 256
HYBRID_MIN_ROWS = 65536
# the dense-head GEMM of tmatmul runs on a side stream beside the tail gather
TMATMUL_HEAD_SIDE_STREAM = True
# its products: f32 (round 6). Alone the bf16x6 form is 30 % faster (1.5 vs 2.0 ms at
# Twitter-World), but beside the tail gather it is starved of CU slots and outlasts the gather
# (9.0 ms in the step's kernel trace): World step 39.09-39.11 -> 38.91-38.98 ms, Twitter-US
# 9.43-9.45 -> 9.35-9.37 with the f32 kernel here (profiles/r06/head_math_ab.txt,
# tools/gpu/head_math.sh). None: dense.TN_MATH.
TMATMUL_HEAD_MATH = "f32"

# Gather hint (round 3, DeviceCSR.gather_hint): on a skewed matrix whose dense operand is far
# larger than the Infinity Cache, the rows of all but the most frequent columns are gathered
# non-temporally so the hot rows (hub nodes) stay cached. Round 4: the hot set comes from the
# graph's own column-frequency histogram -- every column gathered at least GATHER_HINT_MIN_REUSE
# times the mean column count -- capped at GATHER_HINT_HOT_BYTES of rows (the 8 XCDs' L2, 8 x 4
# MiB: hot sets beyond it measured slower); used when the hot set carries >= GATHER_HINT_MIN_SHARE
# of the nonzeros and the operand is >= GATHER_HINT_MIN_TABLE bytes (larger than the cache).
# Measured on the power-law graphs, K = 300 (tools/exp_hot_cold.py, interleaved): World hot sets
# of 8 / 16 / 32 / 64 MiB 6.52 / 6.31 / 6.22 / 6.27 ms vs 6.48 without (4 x the mean count
# reaches 45 MiB there: capped at 32), Twitter-US 1.60 / 1.565 / 1.57 / 1.61 vs 1.667 (4 x the
# mean: 15.5 MiB); every row non-temporal 7.71 vs 6.54; the uniform graphs have no column at
# 4 x the mean (no hint). K = 256: 4.96 (16 MB) / 5.10 (32 MB) vs 5.36 ms, K = 128: 2.36 vs 2.43.
GATHER_HINT = True
# The plan of 'ordered' launches: 1 (whole-workgroup hub rows cut into two column slices on two
# CUs, spmm.hip coop_slice) or 2 (every whole-workgroup row on one CU).
ORDERED_PLAN = 1
GATHER_HINT_HOT_BYTES = 32 << 20
GATHER_HINT_MIN_REUSE = 4.0
GATHER_HINT_MIN_SHARE = 0.25
GATHER_HINT_MIN_TABLE = 256 << 20  # the Infinity Cache (US K = 256, 460 MB: 1.314 -> 1.266 ms)


# Integer ids of operators and row lists, for the registered torch ops (graphconvgeo_amd.ops):
# a custom op takes tensors and scalars only, so gcg::spmm_csr names its DeviceCSR / RowSelection
# by the id given here at construction. Weak: the registry never keeps an operator alive.
_OBJECTS: "weakref.WeakValueDictionary" = weakref.WeakValueDictionary()
_NEXT_ID = itertools.count(1)


def _register_object(obj) -> int:
    i = next(_NEXT_ID)
    _OBJECTS[i] = obj
    return i


def registered(op_id: int):
    """The DeviceCSR / RowSelection registered under op_id (graphconvgeo_amd.ops)."""
    try:
        return _OBJECTS[op_id]
    except KeyError:
        raise KeyError(f"no live sparse operator or row list with id {op_id}") from None


def _stream_handle(device: torch.device) -> C.c_void_p:
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else C.c_void_p(t.data_ptr())


def _require_cuda(t: torch.Tensor, name: str):
    if not t.is_cuda:
        raise ValueError(f"{name} must be a CUDA (HIP) tensor; the graphconvgeo_amd path has "
                         "no CPU fallback")


class RowSelection:
    """A fixed list of output rows (the reference's `target_indices`, mlpconv.py:94).

    Keeps the indices resident as int32 in HBM and carries a content key so the
    launch plan built for it can be cached on the operator.
    """

    def __init__(self, rows, device: Union[str, torch.device] = "cuda"):
        host = np.ascontiguousarray(np.asarray(rows).reshape(-1)).astype(np.int32, copy=False)
        self.host = host
        self.n = int(host.size)
        self.key = hashlib.blake2b(host.tobytes(), digest_size=16).hexdigest() + f":{self.n}"
        self.device_rows = torch.from_numpy(host).to(device)
        self.op_id = _register_object(self)

    def __len__(self):
        return self.n

    def distinct(self):
        """(distinct rows as a RowSelection in increasing order, int64 device index of each
        distinct row's first position, float32 device multiplicities) -- or None when no row
        repeats. A target list drawn with replacement (tensormain.py:226: np.random.choice,
        ~63 % distinct) then costs its distinct rows only: the loss and gradient of a repeated
        target are its multiplicity times one copy's (Theano's inc_subtensor adds the copies,
        mlpconv.py:94). Computed once per selection, on the host."""
        if "_distinct" not in self.__dict__:
            uniq, first, counts = np.unique(self.host, return_index=True, return_counts=True)
            if uniq.size == self.n:
                self._distinct = None
            else:
                dev = self.device_rows.device
                self._distinct = (RowSelection(uniq, dev),
                                  torch.from_numpy(first.astype(np.int64)).to(dev),
                                  torch.from_numpy(counts.astype(np.float32)).to(dev))
        return self._distinct


# Plans released by the garbage collector are destroyed later, at the next plan creation (always
# outside a HIP graph capture: creating a plan synchronizes), never inside __del__: a collection
# can run in the middle of a capture, and hipFree there invalidates it.
_RETIRED_PLANS: list = []


def _destroy_retired_plans():
    while _RETIRED_PLANS:
        h = _RETIRED_PLANS.pop()
        try:
            _native.load().gcg_spmm_plan_destroy(h)
        except Exception:  # interpreter shutdown
            pass


class Plan:
    """Owning wrapper of a gcg_spmm_plan (nnz-balanced task list for one CSR + rows)."""

    def __init__(self, A: "DeviceCSR", rows: Optional[RowSelection], ordered,
                 task_nnz: int):
        _destroy_retired_plans()
        self.A = A
        self.rows = rows
        self.ordered = int(ordered)  # 0 fast, 1 ordered, 2 ordered without column slices
        self.handle = C.c_void_p()
        n_out = rows.n if rows is not None else A.n_rows
        with torch.cuda.device(A.device):
            call("gcg_spmm_plan_create", C.byref(self.handle), A.n_rows, A.n_cols, A.nnz,
                 _ptr(A.indptr), _ptr(rows.device_rows) if rows is not None else None, n_out,
                 int(task_nnz), int(ordered), _stream_handle(A.device))
        self.n_out = n_out
        self._ws = {}

    def info(self) -> dict:
        a, b, c, d = (C.c_int64() for _ in range(4))
        call("gcg_spmm_plan_info", self.handle, C.byref(a), C.byref(b), C.byref(c), C.byref(d))
        e, f, g = (C.c_int64() for _ in range(3))
        call("gcg_spmm_plan_hub_rows", self.handle, C.byref(e), C.byref(f), C.byref(g))
        return {"n_tasks": a.value, "n_long_rows": b.value, "n_segments": c.value,
                "max_task_nnz": d.value, "n_coop_rows": e.value, "n_sliced_rows": f.value,
                "n_slices": g.value}

    def workspace(self, K: int) -> Optional[torch.Tensor]:
        nb = C.c_size_t()
        call("gcg_spmm_plan_workspace_bytes", self.handle, int(K), C.byref(nb))
        if nb.value == 0:
            return None
        ws = self._ws.get(K)
        if ws is None:
            ws = torch.empty((nb.value + 15) // 16 * 4, dtype=torch.float32, device=self.A.device)
            self._ws[K] = ws
        return ws

    def __del__(self):
        h = getattr(self, "handle", None)
        if h is not None and h.value:
            _RETIRED_PLANS.append(h)  # destroyed at the next plan creation (see above)
            self.handle = None


class DeviceCSR:
    """CSR matrix (scipy layout: int32 indptr/indices, float32 data) resident in HBM."""

    def __init__(self, indptr: torch.Tensor, indices: torch.Tensor, data: torch.Tensor,
                 shape, symmetric: Optional[bool] = None, validate: bool = True):
        for t, n in ((indptr, "indptr"), (indices, "indices"), (data, "data")):
            _require_cuda(t, n)
        if indptr.dtype != torch.int32 or indices.dtype != torch.int32:
            raise TypeError("indptr/indices must be int32 (scipy layout for nnz < 2**31)")
        if data.dtype != torch.float32:
            raise TypeError("data must be float32 (mlpconv.py dtype='float32')")
        self.indptr = indptr.contiguous()
        self.indices = indices.contiguous()
        self.data = data.contiguous()
        self.shape = (int(shape[0]), int(shape[1]))
        self.n_rows, self.n_cols = self.shape
        self.nnz = int(self.indices.numel())
        if self.indptr.numel() != self.n_rows + 1 or self.data.numel() != self.nnz:
            raise ValueError("inconsistent CSR arrays")
        self.device = self.indptr.device
        self.symmetric = symmetric
        self._plans = {}
        self._transpose = None
        self.op_id = _register_object(self)
        if validate:
            self.validate()

    # -- construction -------------------------------------------------------------------
    @classmethod
    def from_scipy(cls, m, device: Union[str, torch.device] = "cuda",
                   symmetric: Optional[bool] = None, check_symmetric: bool = False,
                   validate: bool = True) -> "DeviceCSR":
        """Upload a scipy sparse matrix, preserving its storage order (it defines the
        accumulation order and hence the bitwise result, like scipy's csr_matvecs)."""
        if not sps.issparse(m):
            raise ValueError("Input for this layer must be sparse")
        m = m.tocsr() if m.format != "csr" else m
        if m.nnz >= 2**31 or m.shape[0] >= 2**31 - 1:
            raise ValueError("CSR too large for int32 indices")
        dev = torch.device(device)
        if dev.type != "cuda":
            raise ValueError("DeviceCSR lives in HBM: device must be a CUDA (HIP) device")
        if check_symmetric and symmetric is None:
            symmetric = m.shape[0] == m.shape[1] and (abs(m - m.T) > 0).nnz == 0
        indptr = torch.from_numpy(np.ascontiguousarray(m.indptr, dtype=np.int32)).to(dev)
        indices = torch.from_numpy(np.ascontiguousarray(m.indices, dtype=np.int32)).to(dev)
        data = torch.from_numpy(np.ascontiguousarray(m.data, dtype=np.float32)).to(dev)
        return cls(indptr, indices, data, m.shape, symmetric=symmetric, validate=validate)

    def validate(self):
        """Device-side CSR check (monotone indptr, indices in range) -- one sync."""
        status = torch.zeros(1, dtype=torch.int32, device=self.device)
        with torch.cuda.device(self.device):
            call("gcg_csr_validate", self.n_rows, self.n_cols, self.nnz, _ptr(self.indptr),
                 _ptr(self.indices), _ptr(status), _stream_handle(self.device))
        code = int(status.item())
        if code != 0:
            raise ValueError(f"invalid CSR (gcg_status {code}): indptr must be monotone from 0 "
                             "to nnz and every column index in [0, n_cols)")

    def max_row_nnz(self) -> int:
        """Longest row (cached; one device reduction + sync the first time)."""
        if getattr(self, "_max_row_nnz", None) is None:
            self._max_row_nnz = int((self.indptr[1:] - self.indptr[:-1]).max()) if self.n_rows else 0
        return self._max_row_nnz

    def to_scipy(self) -> sps.csr_matrix:
        return sps.csr_matrix((self.data.cpu().numpy(), self.indices.cpu().numpy(),
                               self.indptr.cpu().numpy()), shape=self.shape)

    # -- plans & transpose --------------------------------------------------------------
    def plan(self, rows: Optional[RowSelection] = None, ordered=False,
             task_nnz: int = 0) -> Plan:
        """The launch plan (cached): ordered False / True, or 2 = ordered without column-sliced
        hub rows (gcg_spmm_plan_create; A/B and tests)."""
        key = (rows.key if rows is not None else None, int(ordered), int(task_nnz))
        p = self._plans.get(key)
        if p is None:
            p = Plan(self, rows, ordered, task_nnz)
            self._plans[key] = p
        return p

    def transpose(self) -> "DeviceCSR":
        """CSR of A^T built on the device (stable: within a row, entries keep A's order).

        The gradient of S.dot(A, Z) w.r.t. Z is A^T . gz for ANY A (Theano's Dot grad, the
        backward of mlpconv.py:73,90). `symmetric` True (declared by a builder that makes A
        symmetric by construction, graph.normalize_edges_device) returns A itself; None (unknown, the
        default for an uploaded matrix) builds A^T once and checks it against A
        (check_symmetric): when they hold the same entries, A^T is dropped and A is used -- the
        D^-1/2 (A+I) D^-1/2 of tensormain.py:170-180 -- otherwise the built transpose serves
        every backward (the row-normalized D^-1 (A+I) of main.py:451-455)."""
        if self.symmetric:
            return self
        if self.symmetric is None and self.n_rows == self.n_cols:
            return self if self.check_symmetric() else self._transpose
        if self._transpose is None:
            out_indptr = torch.empty(self.n_cols + 1, dtype=torch.int32, device=self.device)
            out_indices = torch.empty(self.nnz, dtype=torch.int32, device=self.device)
            out_vals = torch.empty(self.nnz, dtype=torch.float32, device=self.device)
            need = C.c_size_t()
            stream = _stream_handle(self.device)
            with torch.cuda.device(self.device):
                call("gcg_csr_transpose_f32", self.n_rows, self.n_cols, self.nnz, None, None, None,
                     None, None, None, None, 0, C.byref(need), stream)
                ws = torch.empty(max(need.value, 1), dtype=torch.uint8, device=self.device)
                call("gcg_csr_transpose_f32", self.n_rows, self.n_cols, self.nnz,
                     _ptr(self.indptr), _ptr(self.indices), _ptr(self.data), _ptr(out_indptr),
                     _ptr(out_indices), _ptr(out_vals), _ptr(ws), need.value, None, stream)
            t = DeviceCSR(out_indptr, out_indices, out_vals, (self.n_cols, self.n_rows),
                          validate=False)
            t._transpose = self
            self._transpose = t
        return self._transpose

    def check_symmetric(self) -> bool:
        """Is A == A^T? Decided once on the device and stored in `symmetric`: A^T is built
        (gcg_csr_transpose_f32) and compared with A -- the CSR arrays bit for bit (a canonical,
        sorted symmetric matrix transposes to the same arrays), else the (row, column, value
        bits) multisets, so a symmetric matrix in any storage order is recognised. Duplicate
        entries must match one for one; a matrix symmetric only after summing its duplicates is
        reported unsymmetric (then its exact transpose is used: still correct). One host sync."""
        if self.symmetric is not None:
            return bool(self.symmetric)
        if self.n_rows != self.n_cols:
            self.symmetric = False
            return False
        self.symmetric = False  # transpose() below builds A^T
        T = self.transpose()
        same = (torch.equal(self.indptr, T.indptr) and torch.equal(self.indices, T.indices)
                and torch.equal(self.data.view(torch.int32), T.data.view(torch.int32))) \
            or self._same_entries(T)
        if same:
            self.symmetric = True
            T._transpose = None
            self._transpose = None
        return same

    def _sorted_entries(self):
        """(row * n_cols + column, value bits) of every entry, sorted by both."""
        lens = (self.indptr[1:] - self.indptr[:-1]).to(torch.int64)
        row = torch.repeat_interleave(torch.arange(self.n_rows, device=self.device), lens,
                                      output_size=self.nnz)
        key = row * self.n_cols + self.indices.to(torch.int64)
        bits = self.data.view(torch.int32)
        o1 = torch.sort(bits, stable=True).indices
        o2 = torch.sort(key[o1], stable=True).indices
        order = o1[o2]
        return key[order], bits[order]

    def _same_entries(self, other: "DeviceCSR") -> bool:
        if self.shape != other.shape or self.nnz != other.nnz:
            return False
        ka, va = self._sorted_entries()
        kb, vb = other._sorted_entries()
        return torch.equal(ka, kb) and torch.equal(va, vb)

    def rows_transpose(self, rows: RowSelection) -> "DeviceCSR":
        """CSR of (A[rows])^T, built on the device once per row list and cached: the operator
        of the gradient of A[rows] . Z w.r.t. Z. Row j lists, in target order, every target
        position p whose row rows[p] holds column j -- duplicated targets stay separate entries
        (tensormain.py:226 draws with replacement). One SpMM with it replaces the scatter-add
        of the row gradient into an N-row zero matrix followed by a full A^T SpMM: it touches
        sum(row lengths of the targets) nonzeros instead of nnz(A), and no N-row temporary."""
        cache = self.__dict__.setdefault("_rows_t", {})
        t = cache.get(rows.key)
        if t is None:
            idx = rows.device_rows.to(torch.int64)
            starts = self.indptr.to(torch.int64)[idx]
            lens = self.indptr.to(torch.int64)[idx + 1] - starts
            indptr = torch.zeros(rows.n + 1, dtype=torch.int64, device=self.device)
            torch.cumsum(lens, 0, out=indptr[1:])
            nnz = int(indptr[-1])
            if nnz >= 2**31:
                raise ValueError("A[rows] has too many nonzeros for int32 CSR")
            owner = torch.repeat_interleave(torch.arange(rows.n, device=self.device), lens,
                                            output_size=nnz)
            src = starts[owner] + torch.arange(nnz, device=self.device) - indptr[owner]
            gathered = DeviceCSR(indptr.to(torch.int32), self.indices[src], self.data[src],
                                 (rows.n, self.n_cols), validate=False)
            t = gathered.transpose()  # stable: within a row of the transpose, target order
            t._transpose = None  # do not pin the gathered copy
            cache[rows.key] = t
        return t

    def gather_hint(self, row_bytes: int) -> Optional[torch.Tensor]:
        """Column indices with bit 31 set on the cold columns (gcg_spmm_csr_f32_planned_hint),
        or None where the hint does not pay (see GATHER_HINT_*). Built once per row size on the
        device (one host sync); the SpMM result does not depend on it (cache policy only). A
        first call inside a HIP-graph capture cannot sync: it returns None (the captured launch
        then gathers every row with the default policy -- same result) without caching."""
        if not GATHER_HINT or self.nnz == 0:
            return None
        n_cap = max(1, GATHER_HINT_HOT_BYTES // max(1, row_bytes))
        if n_cap >= self.n_cols or self.n_cols * row_bytes < GATHER_HINT_MIN_TABLE:
            return None
        cache = self.__dict__.setdefault("_gather_hints", {})
        if n_cap not in cache:
            if torch.cuda.is_current_stream_capturing():
                return None
            idx = self.indices.to(torch.int64)
            counts = torch.bincount(idx, minlength=self.n_cols)
            vals, top = torch.topk(counts, n_cap, sorted=True)
            thr = GATHER_HINT_MIN_REUSE * self.nnz / self.n_cols
            n_hot = int((vals >= thr).sum())
            hint = None
            if n_hot and float(vals[:n_hot].sum()) >= GATHER_HINT_MIN_SHARE * self.nnz:
                hot = torch.zeros(self.n_cols, dtype=torch.bool, device=self.device)
                hot[top[:n_hot]] = True
                cold_bit = torch.tensor(-2 ** 31, dtype=torch.int32, device=self.device)
                hint = torch.where(hot[idx], self.indices, self.indices | cold_bit)
            del idx, counts
            self._hint_hot_rows = n_hot
            cache[n_cap] = hint
        return cache[n_cap]

    def _dense_column_split(self):
        """The columns dense enough that A^T . G is cheaper as a dense MFMA product.

        A bag-of-words X (data.py:378-397) has Zipf column frequencies: a few hundred words
        carry about half the nonzeros. In X^T . G (the W1 gradient, grad of mlpconv.py:71)
        every nonzero gathers one K-wide row of G from HBM (~200 ps per nonzero at
        Twitter-World), while X_head^T . G on the split-K MFMA GEMM streams G once and costs
        ~10-20 ps per (row, column) element -- so columns with density >= HYBRID_MIN_DENSITY
        (at most HYBRID_MAX_COLS of them, the most frequent) move to a dense N x Fh block and
        the rest stay a CSR gather. Built once per matrix on the device; None if no column
        qualifies (H: its densest column is a hub at <= 1 % of N)."""
        if "_dense_split" in self.__dict__:
            return self._dense_split
        split = None
        n, F = self.shape
        thr = max(1, int(np.ceil(HYBRID_MIN_DENSITY * n)))
        if self.nnz and n >= HYBRID_MIN_ROWS:
            cols64 = self.indices.to(torch.int64)
            counts = torch.bincount(cols64, minlength=F)
            q = int((counts >= thr).sum())
            if q:
                # the GEMM computes columns in groups of 64 anyway: fill the last group with
                # the next most frequent columns (free in the GEMM, fewer gathered nonzeros)
                fh = min((q + 63) // 64 * 64, HYBRID_MAX_COLS, F)
                cand = torch.topk(counts, fh, sorted=False).indices
                cand = torch.sort(cand).values
                slot = torch.full((F,), -1, dtype=torch.int64, device=self.device)
                slot[cand] = torch.arange(fh, device=self.device)
                s = slot[cols64]
                del cols64
                head = s >= 0
                lens = (self.indptr[1:] - self.indptr[:-1]).to(torch.int64)
                row = torch.repeat_interleave(torch.arange(n, device=self.device), lens,
                                              output_size=self.nnz)
                Xh = empty_dense(n, fh, self.device)
                Xh.zero_()
                Xh[row[head], s[head]] = self.data[head]
                del row, s
                keep = ~head
                c = torch.zeros(self.nnz + 1, dtype=torch.int64, device=self.device)
                torch.cumsum(keep, 0, out=c[1:])
                tail = DeviceCSR(c[self.indptr.to(torch.int64)].to(torch.int32),
                                 self.indices[keep], self.data[keep], self.shape, validate=False)
                split = (cand, Xh, tail.transpose())
                tail._transpose = None
        self._dense_split = split
        return split

    def tmatmul(self, G: torch.Tensor, mode: str = "auto",
                out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """A^T . G (the gradient of S.dot(A, Z) w.r.t. Z). 'rowwise' / 'ordered' (and 'auto'
        wherever the transpose would run bitwise) gather through CSR(A^T); otherwise the
        dense columns of A go through the MFMA GEMM (_dense_column_split): within fp32
        rounding of the gather (a different summation order), not bitwise."""
        T = self.transpose()
        use_split = mode == "fast" or (
            mode == "auto" and T.max_row_nnz() * TMATMUL_SPLIT_RATIO > max(T.nnz, 1))
        split = self._dense_column_split() if use_split else None
        if split is None:
            return spmm(T, G, mode=mode, out=out)
        from . import dense
        cols, Xh, tail_t = split
        G = _check_dense(G, tail_t)
        # the MFMA head product X_head^T . G (Fh x K: Fh <= 256 in 64-row bands, so the
        # split-K kernel stacks Fh/64 waves along it, round 3: 1.87 ms at Twitter-World, was
        # 2.5 ms as (G^T . X_head)^T) on a side stream, overlapping the HBM-bound tail gather
        main = torch.cuda.current_stream(self.device)
        side = dense._side_stream(self.device) if TMATMUL_HEAD_SIDE_STREAM else main
        side.wait_stream(main)
        with torch.cuda.stream(side):
            G.record_stream(side)  # G (main-stream memory) is read on the side stream
            head = dense.gemm_tn(Xh, G, math=TMATMUL_HEAD_MATH)
            head.record_stream(main)  # side-stream memory, read by the index_copy below
        out = spmm(tail_t, G, mode=mode, out=out)
        main.wait_stream(side)
        out.index_copy_(0, cols, head)
        return out

    def __repr__(self):
        return f"DeviceCSR(shape={self.shape}, nnz={self.nnz}, device={self.device})"


def _same_device(t: torch.Tensor, A: "DeviceCSR", name: str):
    if t.device != A.device:
        raise ValueError(f"{name} is on {t.device} but the operator lives on {A.device}")


def _check_dense(Z: torch.Tensor, A: DeviceCSR):
    _require_cuda(Z, "Z")
    _same_device(Z, A, "Z")
    if Z.dtype != torch.float32:
        raise TypeError(f"Z must be float32, got {Z.dtype}")
    if Z.dim() != 2 or Z.shape[0] != A.n_cols:
        raise ValueError(f"shape mismatch: A is {A.shape}, Z is {tuple(Z.shape)}")
    if Z.stride(1) != 1 and Z.shape[1] > 1:
        Z = Z.contiguous()
    return Z


def _gathers_vec4(Z, ldz: int, Y, ldy: int, K: int, bias) -> bool:
    """Whether the SpMM launch gathers 16-B vectors (spmm.hip pick_vec): ldz, ldy multiples of
    4 floats, 16-B aligned Z / Y / bias. Since round 4 any K (a masked last vector when
    K % 4 != 0). The layout alone decides it (round 5: no environment knob -- ADVICE r04)."""
    del K
    if ldz % 4 or ldy % 4 or Z.data_ptr() % 16 or Y.data_ptr() % 16:
        return False
    return bias is None or bias.data_ptr() % 16 == 0


WIDE_ROW_ALIGN = True  # row_stride: 256-B aligned rows above 512 floats (False: round-3 rule, A/B)


def row_stride(k: int) -> int:
    """Row stride (floats) of empty_dense's k-column rows: a multiple of 4 (16-B aligned rows,
    dwordx4 loads / stores whatever k is), and among those the smallest whose row starts keep a
    gathered row on the fewest 128-B lines. A k = 300 row (1200 B, at least 10 lines) at
    stride 300 starts at 16-B steps into a line and spans 10.25 lines on average; at stride
    304 (1216 B) every row starts 0 or 64 B into a line and spans exactly 10. Strides that are
    a multiple of 128 B (all rows on one alignment) are skipped: 1280-B rows measured slower
    than 1200-B ones (HBM channel interleave). Measured, World H.Z at K = 300: 6.84 -> 6.67-6.70
    ms power-law, 9.37 -> 9.20-9.22 ms uniform (tools/gpu/ld_sweep.sh).
    When no such stride exists within +32 floats (the first line's slack is too small: K = 500,
    1500, the reference's default and tuned hidden sizes, tensormain.py:82,398), the next
    multiple of 128 B puts every row on the minimal line count instead (round 3,
    tools/exp_ld_k.py, World power-law / uniform): K = 500 at 512 floats 11.74 -> 10.99 /
    16.14 -> 14.77 ms, K = 1500 at 1504 33.39 -> 31.89 / 44.18 -> 42.11 ms.
    Rows wider than one 512-float column panel (round 4): the next multiple of 256 B when that
    pads at most 1/12 of the row -- every gathered row then starts on a 256-B boundary, which a
    random gather rewards beyond the line count (World uniform / power-law, interleaved on one
    box, tools/exp_ld_k.py, profiles/r04/ld_sweep.jsonl): C = 930 at 960 floats 30.3 -> 28.2 /
    20.18 -> 20.12 ms (at 932 every row already sat on the minimal 30 lines), K = 600 at 640
    19.87 -> 18.13 / 14.03 -> 13.99, K = 1000 at 1024 32.8 -> 30.4 / 21.5 -> 20.95, K = 1500
    at 1536 45.2 -> 40.7 / 31.0 -> 31.4 ms. At K <= 512 the 256-B strides measured slower
    (K = 129 at 160, 258 at 288) or box-dependent (K = 300 at 320: power-law -1.6 % / +0.9 %)."""
    k4 = (k + 3) // 4 * 4
    if k > 512 and WIDE_ROW_ALIGN:
        k64 = (k + 63) // 64 * 64
        if 12 * (k64 - k) <= k:
            return k64
    if k < 32 or (4 * k) % 128 == 0:
        return k4
    slack = 128 * (-(-4 * k // 128)) - 4 * k  # bytes a row may start into its first line
    for ld in range(k4, k4 + 32, 4):
        step = (4 * ld) % 128
        if step and 128 - math.gcd(step, 128) <= slack:  # row starts: multiples of gcd
            return ld
    return (k + 31) // 32 * 32  # 128-B aligned rows: every row on the minimal line count


def empty_dense(n: int, k: int, device, pad_to: int = 4) -> torch.Tensor:
    """[n, k] float32 view of an [n, ld] buffer, ld = row_stride(k) (pad_to = 4) or k rounded
    up to pad_to: rows 16-B aligned, so the kernels can use dwordx4 loads/stores whatever K
    is, and gathered rows span the fewest 128-B lines."""
    if k <= 0:
        ld = 0
    elif pad_to == 4:
        ld = row_stride(k)
    else:
        ld = (k + pad_to - 1) // pad_to * pad_to
    buf = torch.empty((n, ld), dtype=torch.float32, device=device)
    return buf[:, :k] if ld != k else buf


def empty_gate(n: int, k: int, device) -> torch.Tensor:
    """[n, k] uint8 view of an [n, round4(k)] buffer: the rectify gate of spmm(gate=...)."""
    ld = (k + 3) // 4 * 4
    buf = torch.empty((n, ld), dtype=torch.uint8, device=device)
    return buf[:, :k] if ld != k else buf


def spmm(A: DeviceCSR, Z: torch.Tensor, bias: Optional[torch.Tensor] = None,
         act: Optional[str] = None, rows=None, mode: str = "auto",
         out: Optional[torch.Tensor] = None, task_nnz: int = 0,
         gate: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Y = act(A . Z + bias)[rows] on the GPU (S.dot of mlpconv.py:71,73,90 + epilogue).

    mode  'auto'    : 'ordered' unless the longest row could outlast the launch, then 'fast';
                      'rowwise' on large graphs without hub rows (resolve_auto)
          'fast'    : planned; rows longer than task_nnz split across waves (|err| <= 1e-5)
          'ordered' : planned, rows never split -> bitwise scipy float32
          'rowwise' : plan-less, one wave per output row -> bitwise scipy float32
    rows : None | RowSelection | int array -- output row subset (target_indices).
           A plain array/tensor runs plan-less (no plan to cache).
    gate : optional uint8 [n_out, K] (empty_gate) receiving the rectify gate 2/1/0 of every
           pre-activation (> 0, == 0, < 0) for Theano's rectify gradient (act='relu' only).
    """
    if not isinstance(A, DeviceCSR):
        raise ValueError("Input for this layer must be sparse")
    if mode not in MODES:
        raise ValueError(f"mode must be one of {MODES}")
    if act not in ACTS:
        raise ValueError(f"unsupported activation {act!r}")
    Z = _check_dense(Z, A)
    K = Z.shape[1]
    sel = None
    rows_dev = None
    if rows is not None:
        if isinstance(rows, RowSelection):
            sel = rows
        elif isinstance(rows, torch.Tensor) and rows.is_cuda:
            _same_device(rows, A, "rows")
            rows_dev = rows.to(torch.int32).contiguous()
            mode = "rowwise"
            if rows_dev.numel() and (int(rows_dev.min()) < 0 or int(rows_dev.max()) >= A.n_rows):
                raise IndexError("rows out of range")
        else:
            sel = RowSelection(rows, device=A.device)
        if sel is not None:
            if sel.n and (int(sel.host.min()) < 0 or int(sel.host.max()) >= A.n_rows):
                raise IndexError("rows out of range")
            rows_dev = sel.device_rows
    n_out = A.n_rows if rows_dev is None else int(rows_dev.numel())
    if bias is not None:
        _require_cuda(bias, "bias")
        _same_device(bias, A, "bias")
        if bias.dtype != torch.float32 or bias.numel() != K:
            raise ValueError(f"bias must be float32[{K}]")
        bias = bias.contiguous()
    if out is None:
        out = empty_dense(n_out, K, A.device)
    else:
        _require_cuda(out, "out")
        _same_device(out, A, "out")
        if out.shape != (n_out, K) or out.dtype != torch.float32 or (K > 1 and out.stride(1) != 1):
            raise ValueError(f"out must be float32 [{n_out}, {K}] with unit column stride")
    ldg = 0
    if gate is not None:
        _require_cuda(gate, "gate")
        _same_device(gate, A, "gate")
        if ACTS[act] != GCG_ACT_RELU:
            raise ValueError("gate needs act='relu'")
        if gate.dtype != torch.uint8 or gate.shape != (n_out, K) or (K > 1 and gate.stride(1) != 1):
            raise ValueError(f"gate must be uint8 [{n_out}, {K}] with unit column stride")
        ldg = gate.stride(0) if n_out > 1 else (K + 3) // 4 * 4
        if ldg % 4 or gate.data_ptr() % 4:
            raise ValueError("gate needs a 4-B aligned base and row stride % 4 == 0 (empty_gate)")
    if n_out == 0 or K == 0:
        return out
    ldz = Z.stride(0) if Z.shape[0] > 1 else max(K, 1)
    ldy = out.stride(0) if n_out > 1 else max(K, 1)
    stream = _stream_handle(A.device)
    actc = ACTS[act]
    if mode == "auto":
        mode = resolve_auto(A)
    with torch.cuda.device(A.device):
        if mode == "rowwise":
            call("gcg_spmm_csr_f32_gate", A.n_rows, A.n_cols, A.nnz, _ptr(A.indptr),
                 _ptr(A.indices), _ptr(A.data), _ptr(Z), ldz, K, _ptr(out), ldy, _ptr(bias), actc,
                 _ptr(rows_dev), n_out, _ptr(gate), ldg, stream)
        else:
            plan = A.plan(sel, ordered=ORDERED_PLAN if mode == "ordered" else 0,
                          task_nnz=task_nnz)
            ws = plan.workspace(K)
            # the hint is read by the dwordx4 launches only (spmm.hip pick_vec): never built
            # or looked up for a call that gathers narrower vectors
            hint = A.gather_hint(4 * min(ldz, 512)) if _gathers_vec4(Z, ldz, out, ldy, K, bias) \
                else None
            call("gcg_spmm_csr_f32_planned_hint", plan.handle, _ptr(A.indptr), _ptr(A.indices),
                 _ptr(A.data), _ptr(Z), ldz, K, _ptr(out), ldy, _ptr(bias), actc, _ptr(gate), ldg,
                 _ptr(ws), 0 if ws is None else ws.numel() * 4, _ptr(hint), stream)
    return out


_RELU_WS: dict = {}


def _colsum_workspace(M: int, K: int, device) -> torch.Tensor:
    """Partial-sum workspace of gcg_relu_backward_f32 / gcg_column_sum_f32, per stream."""
    nb = C.c_size_t()
    call("gcg_relu_backward_f32_workspace_bytes", M, K, C.byref(nb))
    key = (device, torch.cuda.current_stream(device).cuda_stream)
    ws = _RELU_WS.get(key)
    if ws is None or ws.numel() * 4 < nb.value:
        ws = torch.empty(max((nb.value + 3) // 4, 1), dtype=torch.float32, device=device)
        _RELU_WS[key] = ws
    return ws


def column_sum(X: torch.Tensor) -> torch.Tensor:
    """X.sum(0) for an M x K float32 matrix (K <= 1024), deterministic (gcg_column_sum_f32):
    the bias gradients (colsum of the logits / pre-activation gradient)."""
    _require_cuda(X, "X")
    M, K = X.shape
    if K > 1 and X.stride(1) != 1:
        X = X.contiguous()
    if K > 256 and M > 1 and (X.stride(0) % 4 or X.data_ptr() % 16):
        X = empty_dense(M, K, X.device).copy_(X)
    out = torch.empty(K, dtype=torch.float32, device=X.device)
    ws = _colsum_workspace(M, K, X.device)
    with torch.cuda.device(X.device):
        call("gcg_column_sum_f32", M, K, _ptr(X), X.stride(0) if M > 1 else K, _ptr(out), _ptr(ws),
             ws.numel() * 4, _stream_handle(X.device))
    return out


def relu_backward(gY: torch.Tensor, Y: Optional[torch.Tensor] = None,
                  out: Optional[torch.Tensor] = None, bias_grad: bool = True,
                  gate: Optional[torch.Tensor] = None):
    """(g, db) and db = column sums of g, one pass (the grad of rectify(. + b),
    mlpconv.py:75-77). With `gate` (the bytes spmm(gate=...) wrote): Theano's rule
    g = gY, gY/2, 0 for a pre-activation > 0, == 0, < 0 (gcg_relu_backward_gate_f32);
    with Y only: g = gY where Y > 0 else 0 (gcg_relu_backward_f32). out may be gY."""
    _require_cuda(gY, "gY")
    M, K = gY.shape
    if gate is not None:
        _require_cuda(gate, "gate")
        if gate.dtype != torch.uint8 or gate.shape != (M, K) or (K > 1 and gate.stride(1) != 1):
            raise ValueError("gate must be uint8 [M, K] with unit column stride")
        ldgate = gate.stride(0) if M > 1 else (K + 3) // 4 * 4
        if ldgate % 4 or gate.data_ptr() % 4:
            raise ValueError("gate needs a 4-B aligned base and row stride % 4 == 0")
        Y = gY  # shape/stride checks below apply to the gradient only
    _require_cuda(Y, "Y")
    if Y.shape != (M, K):
        raise ValueError("gY and Y must have the same shape")
    if out is None:
        out = empty_dense(M, K, gY.device)
    db = torch.empty(K, dtype=torch.float32, device=gY.device) if bias_grad else None
    ws = _colsum_workspace(M, K, gY.device)

    def ld(t):
        return t.stride(0) if t.shape[0] > 1 else K

    def rows16(t):
        return (t.shape[0] <= 1 or t.stride(0) % 4 == 0) and t.data_ptr() % 16 == 0

    if K > 256:  # the wide path loads dwordx4: stage unpadded operands into padded buffers
        if not rows16(gY) or (K > 1 and gY.stride(1) != 1):
            gY = empty_dense(M, K, gY.device).copy_(gY)
        if not rows16(Y) or (K > 1 and Y.stride(1) != 1):
            Y = empty_dense(M, K, Y.device).copy_(Y)
        if not rows16(out):
            raise ValueError("relu_backward: out needs 16-B aligned rows when K > 256")
    for t in (gY, Y, out):
        if K > 1 and t.stride(1) != 1:
            raise ValueError("relu_backward operands need unit column stride")
    with torch.cuda.device(gY.device):
        if gate is not None:
            call("gcg_relu_backward_gate_f32", M, K, _ptr(gY), ld(gY), _ptr(gate), ldgate,
                 _ptr(out), ld(out), _ptr(db), _ptr(ws), ws.numel() * 4, _stream_handle(gY.device))
        else:
            call("gcg_relu_backward_f32", M, K, _ptr(gY), ld(gY), _ptr(Y), ld(Y), _ptr(out),
                 ld(out), _ptr(db), _ptr(ws), ws.numel() * 4, _stream_handle(gY.device))
    return out, db


def index_csr(idx: torch.Tensor, n_rows: int):
    """(seg_ptr, sorted_pos): CSR of an index list, stable (gcg_index_csr)."""
    _require_cuda(idx, "idx")
    idx = idx.to(torch.int32).contiguous()
    n = idx.numel()
    dev = idx.device
    seg_ptr = torch.empty(n_rows + 1, dtype=torch.int32, device=dev)
    sorted_pos = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    need = C.c_size_t()
    stream = _stream_handle(dev)
    with torch.cuda.device(dev):
        call("gcg_index_csr", n, None, n_rows, None, None, None, 0, C.byref(need), stream)
        ws = torch.empty(max(need.value, 1), dtype=torch.uint8, device=dev)
        call("gcg_index_csr", n, _ptr(idx), n_rows, _ptr(seg_ptr), _ptr(sorted_pos), _ptr(ws),
             need.value, None, stream)
    return seg_ptr, sorted_pos


def scatter_add_rows(out: torch.Tensor, seg_ptr: torch.Tensor, sorted_pos: torch.Tensor,
                     src: torch.Tensor) -> torch.Tensor:
    """out[idx[i]] += src[i] for all i, duplicates added in increasing i (gcg_scatter_add_rows_f32)."""
    _require_cuda(out, "out")
    _require_cuda(src, "src")
    if src.stride(1) != 1 and src.shape[1] > 1:
        src = src.contiguous()
    n_rows, K = out.shape
    if src.shape[1] != K:
        raise ValueError("width mismatch")
    lds = src.stride(0) if src.shape[0] > 1 else K
    with torch.cuda.device(out.device):
        call("gcg_scatter_add_rows_f32", n_rows, _ptr(seg_ptr), _ptr(sorted_pos), _ptr(src), lds, K,
             _ptr(out), out.stride(0) if n_rows > 1 else K, _stream_handle(out.device))
    return out


SPGEMM_FLAGS = {"expand_sort": 1, "dense_slabs": 2, "compact_temporary": 4}  # gcg_spgemm_ex


def spgemm(A: DeviceCSR, B: DeviceCSR, accumulate_f64: bool = False,
           a_data64: Optional[torch.Tensor] = None, paths=(), chunk_products: int = 0) -> DeviceCSR:
    """C = A . B on the GPU (the input convolution X_conv = H * X, main.py:530).

    a_data64: float64 values of A (the reference's H is float64 there; implies float64
    accumulation). Entries are summed in scipy's csr_matmat order; exact zeros dropped;
    output canonical float32 (= `(H * X).tocsr().astype('float32')`). paths / chunk_products
    force a path of gcg_spgemm_ex (names of SPGEMM_FLAGS; tests): every path, the same C."""
    flags = 0
    for name in paths:
        flags |= SPGEMM_FLAGS[name]
    if not isinstance(A, DeviceCSR) or not isinstance(B, DeviceCSR):
        raise ValueError("spgemm operands must be DeviceCSR")
    if A.n_cols != B.n_rows:
        raise ValueError(f"shape mismatch {A.shape} x {B.shape}")
    dev = A.device
    stream = _stream_handle(dev)
    P = C.c_int64()
    with torch.cuda.device(dev):
        call("gcg_spgemm_products", A.n_rows, A.nnz, _ptr(A.indptr), _ptr(A.indices), B.n_rows,
             _ptr(B.indptr), C.byref(P), stream)
        cap = max(P.value, 1)
        c_ptr = torch.empty(A.n_rows + 1, dtype=torch.int32, device=dev)
        c_idx = torch.empty(cap, dtype=torch.int32, device=dev)
        c_val = torch.empty(cap, dtype=torch.float32, device=dev)
        nnz = torch.zeros(1, dtype=torch.int64, device=dev)
        if a_data64 is not None:
            _require_cuda(a_data64, "a_data64")
            if a_data64.dtype != torch.float64 or a_data64.numel() != A.nnz:
                raise ValueError("a_data64 must be float64[nnz(A)]")
            a_vals, is64, acc64 = a_data64.contiguous(), 1, 1
        else:
            a_vals, is64, acc64 = A.data, 0, int(bool(accumulate_f64))
        call("gcg_spgemm_ex", A.n_rows, A.n_cols, B.n_cols, A.nnz, _ptr(A.indptr),
             _ptr(A.indices), _ptr(a_vals), is64, B.nnz, _ptr(B.indptr), _ptr(B.indices),
             _ptr(B.data), acc64, P.value, _ptr(c_ptr), _ptr(c_idx), _ptr(c_val), _ptr(nnz), flags,
             int(chunk_products), stream)
    m = int(nnz.item())
    # exact-size copies: the capacity-P buffers (products; 2.5x nnz(C) at Twitter-World) go
    # back to the caching allocator and serve the next call instead of staying pinned by C
    with torch.cuda.device(dev):
        return DeviceCSR(c_ptr, c_idx[:m].clone(), c_val[:m].clone(), (A.n_rows, B.n_cols), validate=False)
