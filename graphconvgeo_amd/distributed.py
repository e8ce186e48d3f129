"""1-D row partition of the graph operator across the GPUs of one node.

The reference is single-process (no collectives anywhere). The
multi-GPU form of its hot path: rank p owns a contiguous, nnz-balanced block of rows
of H (and of every N-row dense tensor); before each SpMM the dense operand is
all-gathered over xGMI (RCCL via torch.distributed 'nccl'), then each rank computes
its own output rows Y_p = H_p . Z.

`all_gather_into_tensor` needs equal chunks, so every rank's block is padded to
`block_rows` rows and H_p's column ids are remapped once, at setup, into that padded
gathered layout (global row j of rank q -> q * block_rows + (j - start_q)).
"""
from __future__ import annotations

from typing import Callable, Optional

import numpy as np
import scipy.sparse as sps
import torch
import torch.distributed as dist


def row_partition(indptr: np.ndarray, parts: int, row_cost: int = 2) -> np.ndarray:
    """Contiguous row blocks with ~equal (nnz + row_cost * rows). Returns bounds[parts+1]."""
    indptr = np.asarray(indptr, dtype=np.int64)
    n = indptr.size - 1
    cost = indptr + row_cost * np.arange(n + 1, dtype=np.int64)
    targets = cost[-1] * np.arange(1, parts, dtype=np.float64) / parts
    cuts = np.searchsorted(cost, targets, side="left")
    bounds = np.concatenate([[0], cuts, [n]]).astype(np.int64)
    return np.maximum.accumulate(bounds)


def remap_columns(cols: np.ndarray, bounds: np.ndarray, block_rows: int) -> np.ndarray:
    """Global column id -> row of the padded all-gathered operand."""
    owner = np.searchsorted(bounds, cols, side="right") - 1
    return (owner * block_rows + (cols - bounds[owner])).astype(np.int32)


class RowPartitionedCSR:
    """Rank-local block of H (rows [start, stop)) with columns in gathered-padded layout.

    local_spmm(A_local, Z_full, **kw) defaults to graphconvgeo_amd.sparse.spmm (HIP);
    tests on CPU/gloo inject the oracle instead.
    """

    def __init__(self, H, rank: int, world: int, device, group=None,
                 local_spmm: Optional[Callable] = None, bounds: Optional[np.ndarray] = None):
        H = sps.csr_matrix(H)
        if H.shape[0] != H.shape[1]:
            raise ValueError("row partition expects a square graph operator")
        self.rank, self.world, self.group = rank, world, group
        self.n = H.shape[0]
        self.bounds = row_partition(H.indptr, world) if bounds is None else np.asarray(bounds)
        self.start, self.stop = int(self.bounds[rank]), int(self.bounds[rank + 1])
        self.block_rows = int(np.diff(self.bounds).max()) if world > 0 else 0
        local = H[self.start:self.stop]
        local = sps.csr_matrix((local.data, remap_columns(local.indices, self.bounds, self.block_rows),
                                local.indptr), shape=(self.stop - self.start, world * self.block_rows))
        self.local_host = local
        self.nnz_local = int(local.nnz)
        self.device = torch.device(device)
        if local_spmm is None:
            from .sparse import DeviceCSR, spmm
            self.A = DeviceCSR.from_scipy(local, self.device)
            self._spmm = spmm
        else:
            self.A = local
            self._spmm = local_spmm
        self._gather_buf = {}

    @property
    def n_local(self) -> int:
        return self.stop - self.start

    def local_rows(self, full: np.ndarray) -> np.ndarray:
        return full[self.start:self.stop]

    def gather_buffer(self, K: int) -> torch.Tensor:
        buf = self._gather_buf.get(K)
        if buf is None:
            buf = torch.zeros((self.world * self.block_rows, K), dtype=torch.float32, device=self.device)
            self._gather_buf[K] = buf
        return buf

    def all_gather(self, Z_local: torch.Tensor) -> torch.Tensor:
        """Z_full (padded layout) <- all-gather of every rank's Z rows."""
        K = Z_local.shape[1]
        full = self.gather_buffer(K)
        if Z_local.shape[0] != self.block_rows:
            send = torch.zeros((self.block_rows, K), dtype=Z_local.dtype, device=Z_local.device)
            send[: Z_local.shape[0]] = Z_local
        else:
            send = Z_local.contiguous()
        if self.world == 1:
            full.copy_(send)
        else:
            dist.all_gather_into_tensor(full, send, group=self.group)
        return full

    def spmm(self, Z_local: torch.Tensor, **kw) -> torch.Tensor:
        """Y_local = (H . Z)[start:stop] = H_p . all_gather(Z)."""
        return self._spmm(self.A, self.all_gather(Z_local), **kw)

    # -- pipelined: all-gather of column chunk c+1 overlaps the SpMM of chunk c -----------
    @staticmethod
    def chunk_bounds(K: int, n_chunks: int):
        """Column chunks of ~K/n_chunks, every boundary a multiple of 4 floats (16-B rows)."""
        n_chunks = max(1, min(n_chunks, (K + 3) // 4))
        step = ((K + n_chunks - 1) // n_chunks + 3) // 4 * 4
        b = list(range(0, K, step)) + [K]
        return [(b[i], b[i + 1]) for i in range(len(b) - 1)]

    def _pipe_buffers(self, K: int, n_chunks: int):
        key = ("pipe", K, n_chunks)
        bufs = self._gather_buf.get(key)
        if bufs is None:
            bufs = []
            for c0, c1 in self.chunk_bounds(K, n_chunks):
                w = c1 - c0
                send = torch.zeros((self.block_rows, w), dtype=torch.float32, device=self.device)
                recv = torch.zeros((self.world * self.block_rows, w), dtype=torch.float32,
                                   device=self.device)
                bufs.append((c0, c1, send, recv))
            self._gather_buf[key] = bufs
        return bufs

    def spmm_pipelined(self, Z_local: torch.Tensor, out: torch.Tensor, n_chunks: int = 4,
                       **kw) -> torch.Tensor:
        """Same result as spmm() (bitwise: each output column is computed by the same
        kernel in the same storage order); comm of chunk c+1 hides behind compute of c."""
        K = Z_local.shape[1]
        bufs = self._pipe_buffers(K, n_chunks)
        rows = Z_local.shape[0]
        for c0, c1, send, _recv in bufs:
            send[:rows].copy_(Z_local[:, c0:c1])
        works = [None] * len(bufs)

        def start(i):
            _c0, _c1, send, recv = bufs[i]
            if self.world == 1:
                recv.copy_(send)
            else:
                works[i] = dist.all_gather_into_tensor(recv, send, group=self.group, async_op=True)

        start(0)
        for i, (c0, c1, _send, recv) in enumerate(bufs):
            if i + 1 < len(bufs):
                start(i + 1)
            if works[i] is not None:
                works[i].wait()  # the compute stream waits for this chunk only
            self._spmm(self.A, recv, out=out[:, c0:c1], **kw)
        return out
