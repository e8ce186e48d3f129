"""1-D row partition of the graph operator across the GPUs of one node.

The reference is single-process (no collectives anywhere). The
multi-GPU form of its hot path: rank p owns a contiguous, nnz-balanced block of rows
of H (and of every N-row dense tensor); before each SpMM the dense operand is
all-gathered over xGMI (RCCL via torch.distributed 'nccl'), then each rank computes
its own output rows Y_p = H_p . Z.

Two exchanges, chosen once at setup (`exchange="auto"`):
  * "allgather": `all_gather_into_tensor` of every rank's whole block. It needs equal
    chunks, so blocks are padded to `block_rows` rows and H_p's column ids are remapped
    into that padded gathered layout (global row j of rank q -> q * block_rows + j - start_q).
  * "halo": each rank receives only the remote rows its H_p references (the halo), via
    `all_to_all_single` with per-peer splits. Every rank holds the whole host H, so the
    send/receive lists are computed locally at setup with no communication. Operand layout
    on rank p: [own rows | halo rows of rank 0 | ... ], halo rows sorted by global id, so
    H_p's remote columns map to n_local + searchsorted(halo, col). On a power-law
    Twitter-World graph the halo is 97 / 87 / 69 % of the remote rows at P = 2 / 4 / 8.
  "auto" picks halo when the largest halo fraction over all ranks is below 0.9.
Both are pipelined over column chunks: the exchange of chunk c+1 overlaps the SpMM of
chunk c. Results are bitwise those of the unpartitioned SpMM (same per-row order).
"""
from __future__ import annotations

from typing import Callable, Optional

import numpy as np
import scipy.sparse as sps
import torch
import torch.distributed as dist


# Partition cost model (round 4). A row longer than HUB_ROW_NNZ nonzeros runs on a whole
# workgroup in 'ordered' mode (spmm.hip coop_row, 8 x the 512-nnz task) and is bound by ONE CU's
# gather rate (~19 GB/s for 1216-B rows: 12,189 nonzeros in 0.77 ms), while the bulk of a block
# spreads over every CU: a hub nonzero costs HUB_WEIGHT bulk nonzeros of the block's time.
HUB_ROW_NNZ = 4096
HUB_WEIGHT = 1.0


def row_partition(indptr: np.ndarray, parts: int, row_cost: int = 2,
                  hub_weight: Optional[float] = None, hub_nnz: int = HUB_ROW_NNZ) -> np.ndarray:
    """Contiguous row blocks with ~equal modelled cost: nnz + row_cost * rows, the nonzeros of
    rows longer than hub_nnz weighted by hub_weight (default HUB_WEIGHT). Returns bounds[parts+1]."""
    indptr = np.asarray(indptr, dtype=np.int64)
    n = indptr.size - 1
    w = HUB_WEIGHT if hub_weight is None else float(hub_weight)
    lens = np.diff(indptr).astype(np.float64)
    if w != 1.0:
        lens = np.where(lens > hub_nnz, lens * w, lens)
    cost = np.zeros(n + 1, dtype=np.float64)
    np.cumsum(lens + row_cost, out=cost[1:])
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
                 local_spmm: Optional[Callable] = None, bounds: Optional[np.ndarray] = None,
                 exchange: str = "auto", halo_threshold: float = 0.9):
        H = sps.csr_matrix(H)
        if H.shape[0] != H.shape[1]:
            raise ValueError("row partition expects a square graph operator")
        if exchange not in ("auto", "allgather", "halo"):
            raise ValueError("exchange must be 'auto', 'allgather' or 'halo'")
        self.rank, self.world, self.group = rank, world, group
        self.n = H.shape[0]
        self._indptr_host = H.indptr
        self.bounds = row_partition(H.indptr, world) if bounds is None else np.asarray(bounds)
        self.start, self.stop = int(self.bounds[rank]), int(self.bounds[rank + 1])
        self.block_rows = int(np.diff(self.bounds).max()) if world > 0 else 0
        b = self.bounds
        # halo (remote rows referenced) of every rank's block, sorted global ids
        halos = []
        for q in range(world):
            cols = np.unique(H.indices[H.indptr[b[q]]:H.indptr[b[q + 1]]])
            halos.append(cols[(cols < b[q]) | (cols >= b[q + 1])])
        remote_total = [max(self.n - (b[q + 1] - b[q]), 1) for q in range(world)]
        self.halo_fraction = max((h.size / t for h, t in zip(halos, remote_total)), default=0.0)
        if exchange == "auto":
            exchange = "halo" if self.halo_fraction < halo_threshold else "allgather"
        self.exchange = exchange
        local = H[self.start:self.stop]
        if exchange == "allgather":
            cols = remap_columns(local.indices, self.bounds, self.block_rows)
            ncols = world * self.block_rows
        else:
            halo = halos[rank]
            own = (local.indices >= self.start) & (local.indices < self.stop)
            cols = np.where(own, local.indices - self.start,
                            self.n_local_rows + np.searchsorted(halo, local.indices)).astype(np.int32)
            ncols = self.n_local_rows + halo.size
            # what this rank receives from q, and sends to p (local row ids), rank order
            self.recv_counts = [int(((halo >= b[q]) & (halo < b[q + 1])).sum()) for q in range(world)]
            send = []
            for p_ in range(world):
                h = halos[p_]
                mine = h[(h >= self.start) & (h < self.stop)] - self.start if p_ != rank else h[:0]
                send.append(mine.astype(np.int64))
            self.send_counts = [int(x.size) for x in send]
            self.send_index_host = np.concatenate(send) if send else np.zeros(0, np.int64)
            self.halo_rows = int(halo.size)
        local = sps.csr_matrix((local.data, cols, local.indptr),
                               shape=(self.stop - self.start, ncols))
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
        if exchange == "halo":
            self.send_index = torch.as_tensor(self.send_index_host, device=self.device)

    def resolve_mode(self, mode: str = "auto") -> str:
        """One SpMM mode for every rank and every N: 'auto' is resolved from the WHOLE graph
        (sparse.auto_mode on the global indptr, which every rank holds: no communication), the
        choice the unpartitioned N = 1 SpMM makes -- so a scaling series runs the same
        arithmetic at every N ('ordered' on the World graph: bitwise scipy at every N). What
        each row block alone would pick is kept in `block_modes` (reporting): at N >= 2 the
        World blocks would pick 'fast' for their ~12k-nonzero hub rows, which the ordered plan
        runs on whole workgroups instead (spmm.hip coop_row; at P = 8 1.16 ms vs 0.91 ms
        fast, against an exchange of several ms)."""
        from .sparse import auto_mode
        ip = np.asarray(self._indptr_host, dtype=np.int64)
        b = self.bounds
        self.block_modes = []
        for q in range(self.world):
            lens = np.diff(ip[b[q]:b[q + 1] + 1])
            self.block_modes.append(auto_mode(int(lens.size), int(lens.sum()),
                                              int(lens.max()) if lens.size else 0))
        if mode != "auto":
            return mode
        lens = np.diff(ip)
        return auto_mode(int(lens.size), int(ip[-1]), int(lens.max()) if lens.size else 0)

    @property
    def n_local_rows(self) -> int:
        return int(self.bounds[self.rank + 1] - self.bounds[self.rank])

    @property
    def n_local(self) -> int:
        return self.stop - self.start

    @property
    def local_block_rows(self) -> int:
        """Rows a caller's local Z block must have (padded for all-gather)."""
        return self.block_rows if self.exchange == "allgather" else self.n_local

    def exchange_bytes_per_row(self, K: int) -> int:
        """Bytes this rank receives per SpMM (for reporting)."""
        rows = (self.world - 1) * self.block_rows if self.exchange == "allgather" else self.halo_rows
        return rows * K * 4

    def local_rows(self, full: np.ndarray) -> np.ndarray:
        return full[self.start:self.stop]

    def operand_rows(self) -> int:
        if self.exchange == "allgather":
            return self.world * self.block_rows
        return self.n_local_rows + self.halo_rows

    def gather_buffer(self, K: int) -> torch.Tensor:
        buf = self._gather_buf.get(K)
        if buf is None:
            buf = torch.zeros((self.operand_rows(), K), dtype=torch.float32, device=self.device)
            self._gather_buf[K] = buf
        return buf

    def _halo_exchange(self, Z_local, c0: int, c1: int, operand: torch.Tensor, async_op: bool):
        """operand[:n_local] = own rows; operand[n_local:] <- halo rows of Z[:, c0:c1]."""
        nl = self.n_local_rows
        zc = Z_local[:nl, c0:c1]
        operand[:nl].copy_(zc)
        if self.world == 1:  # every rank must join the collective, even with empty splits
            return operand, None
        send = torch.index_select(zc, 0, self.send_index)
        work = dist.all_to_all_single(operand[nl:], send, output_split_sizes=self.recv_counts,
                                      input_split_sizes=self.send_counts, group=self.group,
                                      async_op=async_op)
        return operand, work

    def all_gather(self, Z_local: torch.Tensor) -> torch.Tensor:
        """The local SpMM operand: all-gathered (padded) Z, or [own rows | halo rows]."""
        K = Z_local.shape[1]
        if self.exchange == "halo":
            return self._halo_exchange(Z_local, 0, K, self.gather_buffer(K), async_op=False)[0]
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
                send = torch.zeros((self.block_rows if self.exchange == "allgather" else 1, w),
                                   dtype=torch.float32, device=self.device)
                recv = torch.zeros((self.operand_rows(), w), dtype=torch.float32, device=self.device)
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
        if self.exchange == "allgather":
            for c0, c1, send, _recv in bufs:
                send[:rows].copy_(Z_local[:, c0:c1])
        works = [None] * len(bufs)

        def start(i):
            c0, c1, send, recv = bufs[i]
            if self.exchange == "halo":
                works[i] = self._halo_exchange(Z_local, c0, c1, recv, async_op=True)[1]
            elif self.world == 1:
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


def feature_partition(K: int, world: int):
    """Column (feature) blocks of the dense width K, boundaries multiples of 4 floats."""
    step = ((K + world - 1) // world + 3) // 4 * 4
    b = [min(K, i * step) for i in range(world + 1)]
    b[-1] = K
    return [(b[i], b[i + 1]) for i in range(world)]


class FeatureParallelSpMM:
    """H replicated on every GPU, the dense operand split by columns: rank p computes
    Y[:, K_p] = H . Z[:, K_p] with no exchange at all. For a graph that fits one GPU's HBM
    (Twitter-World's H is 0.34 GB of 288 GB) this is the communication-free way to spread
    one SpMM; for the GCN it makes the whole first layer exchange-free (Z1[:, K_p] =
    X . W1[:, K_p], rectify is elementwise) and moves the exchange into layer 2's
    reduction over K. Bitwise equal to the single-GPU product (column-local arithmetic)."""

    def __init__(self, H, rank: int, world: int, device, K: int, local_spmm=None):
        self.rank, self.world = rank, world
        self.device = torch.device(device)
        self.bounds = feature_partition(K, world)
        self.c0, self.c1 = self.bounds[rank]
        if local_spmm is None:
            from .sparse import DeviceCSR, spmm
            self.A = DeviceCSR.from_scipy(sps.csr_matrix(H), self.device, symmetric=True)
            self._spmm = spmm
        else:
            self.A = sps.csr_matrix(H)
            self._spmm = local_spmm

    @property
    def width(self) -> int:
        return self.c1 - self.c0

    def spmm(self, Z_cols: torch.Tensor, **kw) -> torch.Tensor:
        return self._spmm(self.A, Z_cols, **kw)
