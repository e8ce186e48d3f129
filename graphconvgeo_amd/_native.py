"""ctypes binding of the C-ABI in include/gcg_spmm.h (libgcg_spmm.so).

This is the same binding a maintainer would add on the reference side (see
INTEGRATION.md): plain pointers and sizes, a hipStream_t, an int status. There is
no fallback: if the library is missing or fails to load, every entry raises.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

from . import _build
from ._build import LIB

GCG_OK = 0
GCG_ACT_NONE = 0
GCG_ACT_RELU = 1

_STATUS_NAMES = {
    0: "GCG_OK", 1: "GCG_ERR_INVALID_ARG", 2: "GCG_ERR_MISALIGNED", 3: "GCG_ERR_HIP",
    4: "GCG_ERR_ALLOC", 5: "GCG_ERR_BAD_CSR", 6: "GCG_ERR_WORKSPACE",
}

_i64 = C.c_int64
_p = C.c_void_p
_pi64 = C.POINTER(C.c_int64)
_psz = C.POINTER(C.c_size_t)

# name -> (restype, argtypes); mirrors include/gcg_spmm.h one to one.
SIGNATURES = {
    "gcg_version": (C.c_char_p, []),
    "gcg_source_hash": (C.c_char_p, []),
    "gcg_last_error": (C.c_char_p, []),
    "gcg_spmm_csr_f32": (C.c_int, [_i64, _i64, _i64, _p, _p, _p, _p, _i64, _i64, _p, _i64, _p,
                                   C.c_int, _p, _i64, _p]),
    "gcg_spmm_plan_create": (C.c_int, [C.POINTER(_p), _i64, _i64, _i64, _p, _p, _i64, _i64,
                                       C.c_int, _p]),
    "gcg_spmm_plan_destroy": (C.c_int, [_p]),
    "gcg_spmm_plan_workspace_bytes": (C.c_int, [_p, _i64, _psz]),
    "gcg_spmm_plan_info": (C.c_int, [_p, _pi64, _pi64, _pi64, _pi64]),
    "gcg_spmm_plan_hub_rows": (C.c_int, [_p, _pi64, _pi64, _pi64]),
    "gcg_spmm_csr_f32_planned": (C.c_int, [_p, _p, _p, _p, _p, _i64, _i64, _p, _i64, _p,
                                           C.c_int, _p, C.c_size_t, _p]),
    "gcg_spmm_csr_f32_gate": (C.c_int, [_i64, _i64, _i64, _p, _p, _p, _p, _i64, _i64, _p, _i64,
                                        _p, C.c_int, _p, _i64, _p, _i64, _p]),
    "gcg_spmm_csr_f32_planned_gate": (C.c_int, [_p, _p, _p, _p, _p, _i64, _i64, _p, _i64, _p,
                                                C.c_int, _p, _i64, _p, C.c_size_t, _p]),
    "gcg_spmm_csr_f32_planned_hint": (C.c_int, [_p, _p, _p, _p, _p, _i64, _i64, _p, _i64, _p,
                                                C.c_int, _p, _i64, _p, C.c_size_t, _p, _p]),
    "gcg_relu_backward_gate_f32": (C.c_int, [_i64, _i64, _p, _i64, _p, _i64, _p, _i64, _p, _p,
                                             C.c_size_t, _p]),
    "gcg_spmm_plan_host": (C.c_int, [_i64, _p, _p, _i64, _i64, C.c_int, _p, _i64, _pi64, _p,
                                     _i64, _pi64, _pi64]),
    "gcg_adam_step_f32": (C.c_int, [_i64, _p, _p, _p, _p, _p, C.c_float, C.c_float, C.c_float,
                                    _p]),
    "gcg_l1l2_penalty_f32": (C.c_int, [_i64, _p, C.c_float, C.c_float, _p, _p, _p, C.c_size_t,
                                       _p]),
    "gcg_l1l2_grad_f32": (C.c_int, [_i64, _p, C.c_float, C.c_float, _p, _p, _p]),
    "gcg_csr_validate": (C.c_int, [_i64, _i64, _i64, _p, _p, _p, _p]),
    "gcg_index_csr": (C.c_int, [_i64, _p, _i64, _p, _p, _p, C.c_size_t, _psz, _p]),
    "gcg_scatter_add_rows_f32": (C.c_int, [_i64, _p, _p, _p, _i64, _i64, _p, _i64, _p]),
    "gcg_relu_backward_f32_workspace_bytes": (C.c_int, [_i64, _i64, _psz]),
    "gcg_column_sum_f32": (C.c_int, [_i64, _i64, _p, _i64, _p, _p, C.c_size_t, _p]),
    "gcg_relu_backward_f32": (C.c_int, [_i64, _i64, _p, _i64, _p, _i64, _p, _i64, _p, _p,
                                        C.c_size_t, _p]),
    "gcg_csr_transpose_f32": (C.c_int, [_i64, _i64, _i64, _p, _p, _p, _p, _p, _p, _p,
                                        C.c_size_t, _psz, _p]),
    "gcg_normalize_adjacency_f32": (C.c_int, [_i64, _i64, _p, _p, C.c_int, _p, _p, _p, _p, _p,
                                              C.c_size_t, _psz, _p, _p]),
    "gcg_project_mention_graph": (C.c_int, [_i64, _i64, _i64, _p, _p, C.c_int, _p, _p, _i64,
                                            _pi64, _p, _p]),
    "gcg_spgemm_products": (C.c_int, [_i64, _i64, _p, _p, _i64, _p, _pi64, _p]),
    "gcg_gemm_f32": (C.c_int, [_i64, _i64, _i64, _p, _i64, _p, _i64, _p, C.c_int, _p, _i64, _p]),
    "gcg_gemm_nt_f32": (C.c_int, [_i64, _i64, _i64, _p, _i64, _p, _i64, _p, C.c_int, _p, _i64,
                                  _p]),
    "gcg_gemm_nt_f32_bf16x6": (C.c_int, [_i64, _i64, _i64, _p, _i64, _p, _i64, _p, C.c_int, _p,
                                         _i64, _p, _i64, _p]),
    "gcg_gemm_nt_bf16x6_workspace": (_i64, [_i64, _i64]),
    "gcg_project_softmax_xent_bf16x6_workspace": (_i64, [_i64, _i64]),
    "gcg_project_softmax_xent_weighted_ws_f32": (C.c_int, [_i64, _i64, _i64, _p, _i64, _p, _i64,
                                                           _p, _p, C.c_float, _p, _p, _i64, _p,
                                                           _p, _p, _p, _i64, _p]),
    "gcg_project_softmax_xent_f32": (C.c_int, [_i64, _i64, _i64, _p, _i64, _p, _i64, _p, _p,
                                               C.c_float, _p, _p, _i64, _p, _p, _p]),
    "gcg_softmax_xent_f32": (C.c_int, [_i64, _i64, _p, _i64, _p, C.c_float, _p, _p, _i64, _p,
                                       _p, _p]),
    "gcg_project_softmax_xent_weighted_f32": (C.c_int, [_i64, _i64, _i64, _p, _i64, _p, _i64, _p,
                                                        _p, C.c_float, _p, _p, _i64, _p, _p, _p,
                                                        _p]),
    "gcg_softmax_xent_weighted_f32": (C.c_int, [_i64, _i64, _p, _i64, _p, C.c_float, _p, _p, _i64,
                                                _p, _p, _p, _p]),
    "gcg_gemm_tn_f32_workspace_bytes": (C.c_int, [_i64, _i64, _i64, _psz]),
    # round 5: the arithmetic (GCG_MATH_*) and the tile are per-call arguments
    "gcg_dense_tile_count": (C.c_int32, [C.c_int32, C.c_int32]),
    "gcg_gemm": (C.c_int, [_i64, _i64, _i64, _p, _i64, _p, _i64, _p, C.c_int, _p, _i64, C.c_int32,
                           C.c_int32, _p]),
    "gcg_gemm_nt": (C.c_int, [_i64, _i64, _i64, _p, _i64, _p, _i64, _p, C.c_int, _p, _i64,
                              C.c_int32, C.c_int32, _p, _i64, _p]),
    "gcg_gemm_nt_workspace": (_i64, [_i64, _i64, C.c_int32]),
    "gcg_project_softmax_xent": (C.c_int, [_i64, _i64, _i64, _p, _i64, _p, _i64, _p, _p,
                                           C.c_float, _p, _p, _i64, _p, _p, _p, C.c_int32,
                                           C.c_int32, _p, _i64, _p]),
    "gcg_project_softmax_xent_workspace": (_i64, [_i64, _i64, C.c_int32]),
    "gcg_gemm_tn_workspace_bytes": (C.c_int, [_i64, _i64, _i64, C.c_int32, C.c_int32, _psz]),
    "gcg_gemm_tn": (C.c_int, [_i64, _i64, _i64, _p, _i64, _p, _i64, _p, _p, _i64, C.c_int32,
                              C.c_int32, _p, C.c_size_t, _p]),
    "gcg_gemm_tn_f32": (C.c_int, [_i64, _i64, _i64, _p, _i64, _p, _i64, _p, _p, _i64, _p,
                                  C.c_size_t, _p]),
    "gcg_spgemm": (C.c_int, [_i64, _i64, _i64, _i64, _p, _p, _p, C.c_int, _i64, _p, _p, _p,
                             C.c_int, _i64, _p, _p, _p, _p, _p]),
    "gcg_spgemm_ex": (C.c_int, [_i64, _i64, _i64, _i64, _p, _p, _p, C.c_int, _i64, _p, _p, _p,
                                C.c_int, _i64, _p, _p, _p, _p, C.c_int32, _i64, _p]),
}

_lock = threading.Lock()
_lib = None


class NativeError(RuntimeError):
    """A C-ABI call returned a non-zero gcg_status."""

    def __init__(self, fn: str, status: int, msg: str):
        self.status = status
        super().__init__(f"{fn} -> {_STATUS_NAMES.get(status, status)}: {msg}")


def lib_path() -> str:
    return os.environ.get("GCG_LIB", LIB)


def load() -> C.CDLL:
    """Load libgcg_spmm.so (fail loudly; never fall back)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            path = lib_path()
            if not os.path.exists(path):
                raise ImportError(
                    f"graphconvgeo_amd native library not found at {path}; run "
                    "`python -m graphconvgeo_amd._build` (or __graft_entry__.build()) first")
            lib = C.CDLL(path, mode=C.RTLD_GLOBAL)
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(lib, name)
                fn.restype = res
                fn.argtypes = args
            _check_fresh(lib, path)
            _lib = lib
    return _lib


def _check_fresh(lib, path: str) -> None:
    """Refuse a library built from other sources than the tree's (a stale binary would make
    every test and bench measure old kernels). GCG_LIB (an explicit library) or
    GCG_ALLOW_STALE=1 skip the check."""
    if "GCG_LIB" in os.environ or os.environ.get("GCG_ALLOW_STALE") == "1":
        return
    try:
        want = _build.source_hash()
    except OSError:  # sources not shipped next to the library: nothing to compare
        return
    got = lib.gcg_source_hash().decode()
    if got != want:
        raise ImportError(
            f"{path} was built from other sources (hash {got}, tree {want}); rebuild with "
            "`python -m graphconvgeo_amd._build` (or __graft_entry__.build())")


def call(name: str, *args) -> None:
    """Call a status-returning entry point; raise NativeError on failure."""
    lib = load()
    st = getattr(lib, name)(*args)
    if st != GCG_OK:
        msg = lib.gcg_last_error().decode(errors="replace")
        raise NativeError(name, st, msg)


def version() -> str:
    return load().gcg_version().decode()
