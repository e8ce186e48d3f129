"""Host-side graph operator construction (reference layer L1, stays on the host).

`normalize_adjacency` restates tensormain.py:168-181 (same computation at
tensormain.py:94-106 and main.py:511-522):

    adj = nx.adjacency_matrix(graph, nodelist=range(N), weight='w')   # binary: the
          # projection at data.py:240-249 adds edges without a 'w' attribute
    adj.setdiag(1)
    d = adj.sum(axis=1);  d^-1/2 with inf -> 0
    H = D^-1/2 * adj * D^-1/2           (float64, then .astype(float32), tensormain.py:221)

`csr_from_edges` is the same operator built directly from an undirected edge list
(what the synthetic benchmark graphs use): identical values, canonical (sorted)
storage order.
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sps


def normalize_csr(adj, dtype=np.float32) -> sps.csr_matrix:
    """H = D^-1/2 (A + I) D^-1/2 from a (binary) adjacency, scipy expression order.

    Mirrors tensormain.py:172-180 with the two fixes modern scipy needs:
    `sp.sqrt/sp.isinf/sp.errstate` are numpy functions, and the product is spelled
    with csr_matrix operands so `*` is a matrix product.
    """
    import warnings

    adj = sps.csr_matrix(adj, copy=True)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", sps.SparseEfficiencyWarning)
        adj.setdiag(1)
    n, m = adj.shape
    diags = np.asarray(adj.sum(axis=1)).flatten()
    with np.errstate(divide="ignore"):
        diags_sqrt = 1.0 / np.sqrt(diags)
    diags_sqrt[np.isinf(diags_sqrt)] = 0
    d = sps.spdiags(diags_sqrt, [0], m, n, format="csr")
    h = d * adj * d
    return sps.csr_matrix(h.astype(np.float64)).astype(dtype)


def normalize_adjacency(graph, n_nodes: int, dtype=np.float32) -> sps.csr_matrix:
    """tensormain.py:170-181 for a networkx graph over nodes 0..n_nodes-1."""
    import networkx as nx

    adj = nx.adjacency_matrix(graph, nodelist=range(n_nodes), weight="w")
    return normalize_csr(adj, dtype=dtype)


def csr_from_edges(n: int, u: np.ndarray, v: np.ndarray, dtype=np.float32,
                   self_loops: bool = True) -> sps.csr_matrix:
    """Symmetric normalized operator from undirected edges (u[i], v[i]), u != v, unique.

    Values are 1/sqrt(d_i) * 1/sqrt(d_j) computed in float64 (d = degree + 1 with the
    self loop, as setdiag(1) gives) and rounded once to `dtype`, exactly the entries the
    reference's float64 D*A*D product holds before `.astype(float32)`.
    Indices are sorted within each row; nnz = 2E + N.
    """
    u = np.asarray(u, dtype=np.int64)
    v = np.asarray(v, dtype=np.int64)
    rows = np.concatenate([u, v] + ([np.arange(n, dtype=np.int64)] if self_loops else []))
    cols = np.concatenate([v, u] + ([np.arange(n, dtype=np.int64)] if self_loops else []))
    key = rows * n + cols
    order = np.argsort(key, kind="stable")
    rows = rows[order]
    cols = cols[order]
    counts = np.bincount(rows, minlength=n)
    indptr = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(counts, out=indptr[1:])
    deg = counts.astype(np.float64)
    with np.errstate(divide="ignore"):
        dinv = 1.0 / np.sqrt(deg)
    dinv[np.isinf(dinv)] = 0
    data = (dinv[rows] * dinv[cols]).astype(dtype)
    idx_t = np.int32 if (n < 2**31 and len(cols) < 2**31) else np.int64
    return sps.csr_matrix((data, cols.astype(idx_t), indptr.astype(idx_t)), shape=(n, n))


def normalize_edges_device(n: int, u, v, device="cuda", self_loops: bool = True):
    """tensormain.py:170-180 on the GPU: undirected edges -> DeviceCSR H (canonical order,
    duplicates collapsed), values bitwise equal to `csr_from_edges` / the reference's
    float64 D*adj*D cast to float32 (gcg_normalize_adjacency_f32). One sync to read nnz."""
    import ctypes as C

    import torch

    from . import sparse as gs
    from ._native import call

    dev = torch.device(device)
    if dev.type != "cuda":
        raise ValueError("normalize_edges_device builds H in HBM: device must be a CUDA (HIP) device")
    ut = torch.as_tensor(np.asarray(u), dtype=torch.int32).to(dev).contiguous()
    vt = torch.as_tensor(np.asarray(v), dtype=torch.int32).to(dev).contiguous()
    if ut.shape != vt.shape:
        raise ValueError("u and v must have the same length")
    e = int(ut.numel())
    cap = 2 * e + (n if self_loops else 0)
    indptr = torch.empty(n + 1, dtype=torch.int32, device=dev)
    indices = torch.empty(max(cap, 1), dtype=torch.int32, device=dev)
    vals = torch.empty(max(cap, 1), dtype=torch.float32, device=dev)
    nnz = torch.zeros(1, dtype=torch.int64, device=dev)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    need = C.c_size_t()
    stream = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    with torch.cuda.device(dev):
        call("gcg_normalize_adjacency_f32", n, e, None, None, int(self_loops), None, None, None,
             None, None, 0, C.byref(need), None, stream)
        ws = torch.empty(max(need.value, 1), dtype=torch.uint8, device=dev)
        call("gcg_normalize_adjacency_f32", n, e, C.c_void_p(ut.data_ptr()), C.c_void_p(vt.data_ptr()),
             int(self_loops), C.c_void_p(indptr.data_ptr()), C.c_void_p(indices.data_ptr()),
             C.c_void_p(vals.data_ptr()), C.c_void_p(nnz.data_ptr()), C.c_void_p(ws.data_ptr()),
             need.value, None, C.c_void_p(status.data_ptr()), stream)
    if int(status.item()) != 0:
        raise ValueError("edge endpoint out of range [0, n)")
    m = int(nnz.item())
    return gs.DeviceCSR(indptr, indices[:m], vals[:m], (n, n), symmetric=True, validate=False)


def normalized_values_f64(H):
    """float64 entries of H = D^-1/2 (A+I) D^-1/2 for a DeviceCSR built by
    normalize_edges_device (d_i = row length): the operator main.py:522 multiplies X by
    before any float32 cast."""
    import torch

    deg = (H.indptr[1:] - H.indptr[:-1]).to(torch.float64)
    dinv = torch.where(deg > 0, 1.0 / torch.sqrt(deg), torch.zeros_like(deg))
    rows = torch.repeat_interleave(torch.arange(H.n_rows, device=H.device),
                                   (H.indptr[1:] - H.indptr[:-1]).long())
    return dinv[rows] * dinv[H.indices.long()]
