"""1-D row partition of the graph operator across the GPUs of one node.

The reference is single-process (no collectives anywhere). The
multi-GPU form of its hot path: rank p owns a contiguous, nnz-balanced block of rows
of H (and of every N-row dense tensor); before each SpMM the dense operand is
all-gathered over xGMI (RCCL via torch.distributed 'nccl'), then each rank computes
its own output rows Y_p = H_p . Z.

Three exchanges, chosen once at setup (`exchange=`), all into one operand layout per rank:
  * "allgather": `all_gather_into_tensor` of every rank's whole block, in place (the rank's
    input is its own slot of the output). It needs equal chunks, so blocks are padded to
    `block_rows` rows and H_p's column ids are remapped into that padded gathered layout
    (global row j of rank q -> q * block_rows + j - start_q).
  * "mesh" (round 4): the same layout filled by one isend + irecv pair per peer in one batch
    (`batch_isend_irecv`): every xGMI link of the fully connected node busy at once, exact row
    counts on the wire -- the direct algorithm SURVEY.md §5 / §8e prefer to a ring.
  * "halo": each rank receives only the remote rows its H_p references (the halo), via
    `all_to_all_single` with per-peer splits. Every rank holds the whole host H, so the
    send/receive lists are computed locally at setup with no communication. Operand layout
    on rank p: [own rows | halo rows of rank 0 | ... ], halo rows sorted by global id, so
    H_p's remote columns map to n_local + searchsorted(halo, col). On a power-law
    Twitter-World graph the halo is 97 / 87 / 69 % of the remote rows at P = 2 / 4 / 8.
  "auto" picks halo when the largest halo fraction over all ranks is below 0.9, else allgather.
All are pipelined over column chunks (count chosen per call, choose_chunks, from every rank's
numbers so that every rank issues the same collectives): every chunk's exchange is issued up
front, chunk c's SpMM waits for its own. A producer may write its rows
straight into the exchange buffers (chunk_buffers(...).own_views()), so the step copies nothing.
Results are bitwise those of the unpartitioned SpMM (same per-row order).

The gradient of a target-row subset (the reference's `[target_indices]`, mlpconv.py:94)
exchanges only the distinct targets' gradient rows (TargetRowsBackward).
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


def host_is_symmetric(H) -> bool:
    """H == H^T for a host CSR (every rank holds H: no communication). A canonical symmetric
    matrix transposes to the same arrays (checked first, linear); otherwise the numeric
    difference decides (duplicates summed)."""
    H = sps.csr_matrix(H)
    if H.shape[0] != H.shape[1]:
        return False
    T = H.T.tocsr()
    if (np.array_equal(H.indptr, T.indptr) and np.array_equal(H.indices, T.indices)
            and np.array_equal(H.data.view(np.uint8), T.data.view(np.uint8))):
        return True
    return (abs(H - T) > 0).nnz == 0


def _same_host_csr(a, b) -> bool:
    a, b = sps.csr_matrix(a), sps.csr_matrix(b)
    if a.indptr is b.indptr and a.indices is b.indices and a.data is b.data:
        return a.shape == b.shape
    return (a.shape == b.shape and a.nnz == b.nnz and np.array_equal(a.indptr, b.indptr)
            and np.array_equal(a.indices, b.indices) and np.array_equal(a.data, b.data))


def remap_columns(cols: np.ndarray, bounds: np.ndarray, block_rows: int) -> np.ndarray:
    """Global column id -> row of the padded all-gathered operand."""
    owner = np.searchsorted(bounds, cols, side="right") - 1
    return (owner * block_rows + (cols - bounds[owner])).astype(np.int32)


# Chunk-count model (round 4, RowPartitionedCSR.choose_chunks). The exchange of column chunk c+1
# overlaps the local SpMM of chunk c; each extra chunk costs the SpMM ~CHUNK_COST (narrower
# gathers: 2 chunks x1.06-1.07, 4 chunks x1.26-1.30, profiles/HISTORY.md §4). Exchange rate: xGMI is a full
# mesh of 7 links per MI355X, ~XGMI_LINK_GBPS each way per link in practice (153.6 GB/s per link
# both ways together), min(P - 1, 7) of them busy; local SpMM at LOCAL_SPMM_GBPS edge-centric.
XGMI_LINK_GBPS = 64.0
LOCAL_SPMM_GBPS = 7000.0
CHUNK_COST = 0.09
MAX_CHUNKS = 4
MIN_CHUNK_COLS = 64

EXCHANGES = ("auto", "allgather", "mesh", "halo")


def _spmm_bytes(n_out: int, nnz: int, k: int) -> int:
    return 4 * (n_out + 1) + 8 * nnz + 4 * k * nnz + 4 * k * n_out


def _wait(work):
    if work is None:
        return
    for w in (work if isinstance(work, (list, tuple)) else (work,)):
        w.wait()


DIST_TIMEOUT_S = 180.0  # a collective stuck this long is a hang (well inside a 600 s job limit)


def init_process_group(backend: str, device=None, timeout_s: float = DIST_TIMEOUT_S):
    """torch.distributed.init_process_group for the row partition, made to fail rather than
    hang: an explicit collective timeout, and (NCCL = RCCL) the async error handling that tears
    the process down with a message when a collective exceeds it, so a stuck first RCCL run
    ends non-zero instead of sitting until the driver's limit."""
    import datetime
    import os
    if backend == "nccl":
        # 1 = abort the communicator and tear the process down on a failed / timed-out
        # collective (the watchdog thread raises; no rank is left waiting)
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        os.environ.setdefault("TORCH_NCCL_DUMP_ON_TIMEOUT", "0")
    kw = {"timeout": datetime.timedelta(seconds=float(timeout_s))}
    if backend == "nccl" and device is not None:
        kw["device_id"] = torch.device(device)
    dist.init_process_group(backend, **kw)
    return dist.group.WORLD


class PartitionPlan:
    """The rank-independent structure of a 1-D row partition of the host H: the bounds, every
    rank's halo (the remote rows its block references, sorted global ids), nonzeros and rows.
    Every rank holds the whole host H, so every rank computes the same plan with no
    communication; a single process building all P ranks (tests, tools) computes it once.
    Decisions that must agree across ranks -- the exchange chosen by 'auto', the column-chunk
    count (RowPartitionedCSR.choose_chunks) -- are taken from it, never from rank-local data."""

    def __init__(self, H, world: int, bounds: Optional[np.ndarray] = None):
        H = sps.csr_matrix(H)
        if H.shape[0] != H.shape[1]:
            raise ValueError("row partition expects a square graph operator")
        self.H, self.world, self.n = H, int(world), H.shape[0]
        self.bounds = row_partition(H.indptr, world) if bounds is None else np.asarray(bounds)
        if self.bounds.size != world + 1:
            raise ValueError("bounds must hold world + 1 entries")
        b = self.bounds
        self.rows = np.diff(b).astype(np.int64)
        self.block_rows = int(self.rows.max()) if world > 0 else 0
        ip = np.asarray(H.indptr, dtype=np.int64)
        self.nnz = (ip[b[1:]] - ip[b[:-1]]).astype(np.int64)
        self.halos = []
        for q in range(world):
            cols = np.unique(H.indices[ip[b[q]]:ip[b[q + 1]]])
            self.halos.append(cols[(cols < b[q]) | (cols >= b[q + 1])].astype(np.int64))
        remote_total = [max(self.n - int(self.rows[q]), 1) for q in range(world)]
        self.halo_fraction = max((h.size / t for h, t in zip(self.halos, remote_total)),
                                 default=0.0)

    def resolve_exchange(self, exchange: str, halo_threshold: float = 0.9) -> str:
        if exchange not in EXCHANGES:
            raise ValueError(f"exchange must be one of {EXCHANGES}")
        if exchange == "auto":
            return "halo" if self.halo_fraction < halo_threshold else "allgather"
        return exchange

    def rows_in(self, exchange: str) -> np.ndarray:
        """Rows every rank receives per exchange (index = rank)."""
        P = self.world
        if exchange == "allgather":
            return np.full(P, (P - 1) * self.block_rows, dtype=np.int64)
        if exchange == "mesh":
            return int(self.rows.sum()) - self.rows
        if exchange == "halo":
            return np.array([h.size for h in self.halos], dtype=np.int64)
        raise ValueError(f"exchange must be one of {EXCHANGES[1:]}")

    def choose_chunks(self, exchange: str, K: int) -> int:
        """Column chunks for one exchange + SpMM of width K, the same on every rank: 1 at world
        1; otherwise the count minimising the SLOWEST rank's pipeline_time (every rank's
        exchange bytes over min(P - 1, 7) xGMI links, every rank's local SpMM estimate), chunks
        >= 64 columns. Every chunk is one collective per rank, so the count must agree: a
        rank-local choice would issue different numbers and widths of collectives."""
        if self.world == 1:
            return 1
        links = min(self.world - 1, 7)
        w4 = (K + 3) // 4 * 4  # the exchange moves the padded width
        t_x = self.rows_in(exchange) * w4 * 4 / (XGMI_LINK_GBPS * 1e9 * links)
        t_s = [_spmm_bytes(int(r), int(z), K) / (LOCAL_SPMM_GBPS * 1e9)
               for r, z in zip(self.rows, self.nnz)]
        cmax = max(1, min(MAX_CHUNKS, K // MIN_CHUNK_COLS))

        def worst(c):
            return max(pipeline_time(float(x), s, c) for x, s in zip(t_x, t_s))
        return min(range(1, cmax + 1), key=lambda c: (worst(c), c))


def _as_ids(src) -> np.ndarray:
    if isinstance(src, tuple):
        return np.arange(src[0], src[1], dtype=np.int64)
    return np.asarray(src, dtype=np.int64)


def pipeline_time(t_exchange: float, t_spmm: float, chunks: int) -> float:
    """Modelled step time of `chunks` column chunks: exchanges back to back on the comm stream,
    chunk i's SpMM after its exchange and after chunk i-1's SpMM."""
    f = 1.0 + CHUNK_COST * (chunks - 1)
    end_x = end_s = 0.0
    for _ in range(chunks):
        end_x += t_exchange / chunks
        end_s = max(end_s, end_x) + t_spmm * f / chunks
    return end_s


class ExchangeLayout:
    """Where every rank's rows sit in a local SpMM's operand, and how they get there.

    "allgather" / "mesh": rank q's rows at [q * pad, q * pad + counts[q]) of a [world * pad, w]
      buffer. allgather = `all_gather_into_tensor` IN PLACE (this rank's input is its own slot of
      the output: no send copy); mesh = one isend + irecv per peer in one batch
      (`batch_isend_irecv`: every xGMI link of the full mesh busy at once, exact row counts, no
      padding on the wire) -- SURVEY.md §5 / §8e prefer a direct mesh to a ring.
    "halo": own rows at [0, n_own), then the remote rows H_p references, grouped by owner
      (`all_to_all_single` with per-peer splits; the send rows are gathered by index_select).
    A producer may write the own rows straight into `own(buf)`: then nothing is copied."""

    def __init__(self, method: str, rank: int, world: int, group=None, counts=None,
                 pad: int = 0, n_own: int = 0, halo_rows: int = 0, send_index=None,
                 send_counts=None, recv_counts=None, sources=None):
        self.method, self.rank, self.world, self.group = method, rank, world, group
        # sources: which global rows each slot holds (operand_ids) -- per rank q the global ids
        # of its block's rows (allgather / mesh: an array or a (start, stop) range), or for
        # halo (own global ids, halo global ids)
        self.sources = sources
        if method in ("allgather", "mesh"):
            self.counts = [int(c) for c in counts]
            self.pad = int(pad)
            self.rows = world * self.pad
            self.own_off, self.n_own = rank * self.pad, self.counts[rank]
        elif method == "halo":
            self.rows = n_own + halo_rows
            self.own_off, self.n_own = 0, n_own
            self.send_index = send_index
            self.send_counts, self.recv_counts = send_counts, recv_counts
        else:
            raise ValueError(f"exchange must be one of {EXCHANGES[1:]}")

    def own(self, buf: torch.Tensor) -> torch.Tensor:
        return buf[self.own_off:self.own_off + self.n_own]

    def operand_ids(self) -> np.ndarray:
        """The global row each operand row holds after an exchange (-1: padding, never
        referenced by the local operator) -- what the exchange must produce, so a single process
        can build any rank's operand from the whole dense matrix (tests, tools)."""
        if self.sources is None:
            raise ValueError("this layout was built without its row sources")
        ids = np.full(self.rows, -1, dtype=np.int64)
        if self.method == "halo":
            own, halo = self.sources
            ids[:self.n_own] = _as_ids(own)
            ids[self.n_own:] = _as_ids(halo)
            return ids
        for q, src in enumerate(self.sources):
            ids[q * self.pad:q * self.pad + self.counts[q]] = _as_ids(src)
        return ids

    def bytes_in(self, width: int) -> int:
        """Bytes this rank receives per exchange of `width` float columns."""
        if self.method == "halo":
            return (self.rows - self.n_own) * width * 4
        if self.method == "allgather":
            return (self.world - 1) * self.pad * width * 4
        return (sum(self.counts) - self.n_own) * width * 4

    def exchange(self, buf: torch.Tensor, async_op: bool = True):
        """Fill `buf`'s remote rows from the other ranks (own rows already in place)."""
        if self.world == 1:
            return None
        if self.method == "allgather":
            own = buf[self.own_off:self.own_off + self.pad]
            return dist.all_gather_into_tensor(buf, own, group=self.group, async_op=async_op)
        if self.method == "mesh":
            mine = buf[self.own_off:self.own_off + self.n_own]
            if buf.is_cuda and dist.get_backend(self.group) == "gloo":
                return self._mesh_gloo_staged(buf, mine)
            ops = []
            for q in range(self.world):
                if q == self.rank:
                    continue
                peer = q if self.group is None else dist.get_global_rank(self.group, q)
                if self.n_own:
                    ops.append(dist.P2POp(dist.isend, mine, peer, self.group))
                if self.counts[q]:
                    ops.append(dist.P2POp(dist.irecv, buf[q * self.pad:q * self.pad + self.counts[q]],
                                          peer, self.group))
            if not ops:
                return None
            works = dist.batch_isend_irecv(ops)
            if not async_op:
                _wait(works)
                return None
            return works
        own = buf[:self.n_own]
        send = torch.index_select(own, 0, self.send_index)
        return dist.all_to_all_single(buf[self.n_own:], send, output_split_sizes=self.recv_counts,
                                      input_split_sizes=self.send_counts, group=self.group,
                                      async_op=async_op)

    def _mesh_gloo_staged(self, buf, mine):
        """The mesh over gloo with device tensors (the one-GPU rehearsal only: gloo's
        point-to-point ops take host memory): the same isend / irecv pairs on host copies,
        completed before returning."""
        host_mine = mine.cpu()
        recv = {q: torch.empty((self.counts[q], buf.shape[1]), dtype=buf.dtype)
                for q in range(self.world) if q != self.rank and self.counts[q]}
        ops = []
        for q in range(self.world):
            if q == self.rank:
                continue
            peer = q if self.group is None else dist.get_global_rank(self.group, q)
            if self.n_own:
                ops.append(dist.P2POp(dist.isend, host_mine, peer, self.group))
            if q in recv:
                ops.append(dist.P2POp(dist.irecv, recv[q], peer, self.group))
        if ops:
            _wait(dist.batch_isend_irecv(ops))
        for q, t in recv.items():
            buf[q * self.pad:q * self.pad + self.counts[q]].copy_(t)
        return None


class _ChunkBuffers:
    """Column-chunk operand buffers of one layout: [(c0, c1, buf [rows, round4(c1 - c0)])],
    padded widths (16-B rows, dwordx4 gathers; the exchange moves the padded width)."""

    def __init__(self, layout: ExchangeLayout, K: int, n_chunks: int, device):
        self.layout = layout
        self.chunks = []
        for c0, c1 in RowPartitionedCSR.chunk_bounds(K, n_chunks):
            w4 = (c1 - c0 + 3) // 4 * 4
            self.chunks.append((c0, c1, torch.zeros((layout.rows, w4), dtype=torch.float32,
                                                    device=device)))

    def own_views(self):
        """The own-rows slot of every chunk, [n_own, c1 - c0] each: a producer writing there
        makes the pipeline copy-free."""
        return [self.layout.own(buf)[:, :c1 - c0] for c0, c1, buf in self.chunks]

    def fill(self, Z_local: torch.Tensor):
        """Copy this rank's rows of Z into every chunk's own slot, unless they are already there."""
        for (c0, c1, buf), own in zip(self.chunks, self.own_views()):
            src = Z_local[:own.shape[0], c0:c1]
            if src.data_ptr() == own.data_ptr() and src.stride() == own.stride():
                continue
            own.copy_(src)


# When a list: every pipelined_product call appends its arguments (measurement tools replay
# the exchanges and the local SpMMs of a step alone). None in normal runs.
TRACE: Optional[list] = None

# When set: a single-process rehearsal of one rank. pipelined_product calls
# LOOPBACK(layout, buf, c0, c1) instead of the collective; the function writes what the exchange
# would deliver into buf's remote rows (layout.operand_ids() names them). tests/
# test_partition_world_gpu.py runs every rank of a P-way partition of the World graph in one
# process this way. None in normal runs.
LOOPBACK: Optional[Callable] = None


def pipelined_product(spmm_into, A, bufs: _ChunkBuffers, out: torch.Tensor, bias=None,
                      gate=None, **kw) -> torch.Tensor:
    """out[:, c0:c1] = spmm(A, exchanged chunk c) for every column chunk, every exchange issued
    up front on the communication stream (chunk c+1's transfer overlaps chunk c's SpMM; the
    compute stream waits for one chunk at a time). Bias and gate are sliced per chunk; every
    output column is computed by the same kernel in the same storage order as unchunked."""
    if TRACE is not None:  # measurement hook (tools/bench_train_dist.py --phases)
        TRACE.append((spmm_into, A, bufs, out, bias, gate, dict(kw)))
    if LOOPBACK is not None:
        works = [LOOPBACK(bufs.layout, buf, c0, c1) for c0, c1, buf in bufs.chunks]
    else:
        works = [bufs.layout.exchange(buf, async_op=True) for _c0, _c1, buf in bufs.chunks]
    for (c0, c1, buf), work in zip(bufs.chunks, works):
        _wait(work)
        spmm_into(A, buf[:, :c1 - c0], out[:, c0:c1],
                  bias=None if bias is None else bias[c0:c1],
                  gate=None if gate is None else gate[:, c0:c1], **kw)
    return out


class RowPartitionedCSR:
    """Rank-local block of H (rows [start, stop)) with columns in the exchange layout.

    local_spmm(A_local, Z_full, **kw) defaults to graphconvgeo_amd.sparse.spmm (HIP);
    tests on CPU/gloo inject the oracle instead (it must take out=, bias=, act=, rows=, gate=).
    """

    def __init__(self, H, rank: int, world: int, device, group=None,
                 local_spmm: Optional[Callable] = None, bounds: Optional[np.ndarray] = None,
                 exchange: str = "auto", halo_threshold: float = 0.9,
                 plan: Optional[PartitionPlan] = None):
        if plan is None:
            plan = PartitionPlan(H, world, bounds)
        elif H is not None and H is not plan.H and not _same_host_csr(H, plan.H):
            raise ValueError("plan was built for another graph (pass H=None with a plan)")
        elif plan.world != world or (bounds is not None and
                                     not np.array_equal(np.asarray(bounds), plan.bounds)):
            raise ValueError("plan was built for another partition")
        H = plan.H
        if not 0 <= rank < world:
            raise ValueError(f"rank {rank} outside world {world}")
        self.plan = plan
        self.rank, self.world, self.group = rank, world, group
        self.n = H.shape[0]
        self._indptr_host = H.indptr
        self.bounds = plan.bounds
        self.start, self.stop = int(self.bounds[rank]), int(self.bounds[rank + 1])
        self.block_rows = plan.block_rows
        b = self.bounds
        halos = plan.halos
        self.halo_fraction = plan.halo_fraction
        exchange = plan.resolve_exchange(exchange, halo_threshold)
        self.exchange = exchange
        local = H[self.start:self.stop]
        self.local_global = local  # global column ids (target-row backward operators)
        self.device = torch.device(device)
        if exchange in ("allgather", "mesh"):
            cols = remap_columns(local.indices, self.bounds, self.block_rows)
            ncols = world * self.block_rows
            self.layout = ExchangeLayout(exchange, rank, world, group, counts=np.diff(self.bounds),
                                         pad=self.block_rows,
                                         sources=[(int(b[q]), int(b[q + 1])) for q in range(world)])
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
            self.send_index = torch.as_tensor(self.send_index_host, device=self.device)
            self.layout = ExchangeLayout("halo", rank, world, group, n_own=self.n_local,
                                         halo_rows=self.halo_rows, send_index=self.send_index,
                                         send_counts=self.send_counts,
                                         recv_counts=self.recv_counts,
                                         sources=((self.start, self.stop), halo))
        local = sps.csr_matrix((local.data, cols, local.indptr),
                               shape=(self.stop - self.start, ncols))
        self.local_host = local
        self.nnz_local = int(local.nnz)
        if local_spmm is None:
            from .sparse import DeviceCSR, spmm
            self.A = DeviceCSR.from_scipy(local, self.device)
            self._spmm = spmm
            self._on_device = True
        else:
            self.A = local
            self._spmm = local_spmm
            self._on_device = False
        self._bufs = {}
        self.chunks_override = None

    def resolve_mode(self, mode: str = "auto") -> str:
        """One SpMM mode for every rank and every N: 'auto' is resolved from the WHOLE graph
        (sparse.auto_mode on the global indptr, which every rank holds: no communication), the
        choice the unpartitioned N = 1 SpMM makes -- so a scaling series runs the same
        arithmetic at every N ('ordered' on the World graph: bitwise scipy at every N). What
        each row block alone would pick is kept in `block_modes` (reporting): at N >= 2 the
        World blocks would pick 'fast' for their ~12k-nonzero hub rows, which the ordered plan
        runs on whole workgroups instead (spmm.hip coop_row; round 4, tools/exp_partition.py:
        the slowest of 8 blocks 1.054 ms, 1.011 x the mean)."""
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
        return self.block_rows if self.exchange in ("allgather", "mesh") else self.n_local

    def exchange_bytes_per_row(self, K: int) -> int:
        """Bytes this rank receives per SpMM of width K (for reporting)."""
        return self.layout.bytes_in(K)

    def local_rows(self, full: np.ndarray) -> np.ndarray:
        return full[self.start:self.stop]

    def operand_rows(self) -> int:
        return self.layout.rows

    # -- chunk count ----------------------------------------------------------------------
    def choose_chunks(self, K: int) -> int:
        """Column chunks for one exchange + SpMM of width K (PartitionPlan.choose_chunks): the
        same count on every rank -- decided from every rank's exchange bytes and local SpMM,
        which every rank derives from the host H -- so all ranks issue the same collectives."""
        return self.plan.choose_chunks(self.exchange, K)

    def _n_chunks(self, n_chunks, K: int) -> int:
        if n_chunks in (None, "auto", 0):  # chunks_override: a fixed count for 'auto' callers
            return self.chunks_override or self.choose_chunks(K)
        return max(1, int(n_chunks))

    # -- operand buffers --------------------------------------------------------------------
    @staticmethod
    def chunk_bounds(K: int, n_chunks: int):
        """Column chunks of ~K/n_chunks, every boundary a multiple of 4 floats (16-B rows)."""
        n_chunks = max(1, min(n_chunks, (K + 3) // 4))
        step = ((K + n_chunks - 1) // n_chunks + 3) // 4 * 4
        b = list(range(0, K, step)) + [K]
        return [(b[i], b[i + 1]) for i in range(len(b) - 1)]

    def chunk_buffers(self, K: int, n_chunks="auto") -> _ChunkBuffers:
        """The exchange operand buffers of width K in n_chunks column chunks (cached). Their
        own_views() are where a producer may write this rank's rows (no staging copy)."""
        c = self._n_chunks(n_chunks, K)
        key = (K, c)
        bufs = self._bufs.get(key)
        if bufs is None:
            bufs = _ChunkBuffers(self.layout, K, c, self.device)
            self._bufs[key] = bufs
        return bufs

    def gather_buffer(self, K: int) -> torch.Tensor:
        return self.chunk_buffers(K, 1).chunks[0][2]

    def all_gather(self, Z_local: torch.Tensor) -> torch.Tensor:
        """The local SpMM operand in one exchange: all-gathered / meshed (padded) Z, or
        [own rows | halo rows]."""
        K = Z_local.shape[1]
        bufs = self.chunk_buffers(K, 1)
        bufs.fill(Z_local)
        buf = bufs.chunks[0][2]
        _wait(self.layout.exchange(buf, async_op=False))
        return buf[:, :K]

    def _spmm_into(self, A, Z, out, **kw):
        kw = {k: v for k, v in kw.items() if v is not None}
        return self._spmm(A, Z, out=out, **kw)

    def spmm(self, Z_local: torch.Tensor, **kw) -> torch.Tensor:
        """Y_local = (H . Z)[start:stop] = H_p . all_gather(Z)."""
        return self._spmm(self.A, self.all_gather(Z_local), **kw)

    # -- pipelined: the exchange of column chunk c+1 overlaps the SpMM of chunk c ------------
    def spmm_pipelined(self, Z_local: Optional[torch.Tensor], out: torch.Tensor,
                       n_chunks="auto", bias=None, gate=None, spmm_into=None, **kw) -> torch.Tensor:
        """Same result as spmm() (bitwise: each output column is computed by the same kernel in
        the same storage order); comm of chunk c+1 hides behind compute of chunk c.
        Z_local None: the producer already wrote this rank's rows into chunk_buffers(K,
        n_chunks).own_views() (no copy at all). World 1: the local SpMM on Z_local itself."""
        spmm_into = spmm_into or self._spmm_into
        K = out.shape[1]
        if self.world == 1 and Z_local is not None:
            return spmm_into(self.A, Z_local[:self.operand_rows()], out, bias=bias, gate=gate, **kw)
        bufs = self.chunk_buffers(K, n_chunks)
        if Z_local is not None:
            bufs.fill(Z_local)
        return pipelined_product(spmm_into, self.A, bufs, out, bias=bias, gate=gate, **kw)

    # -- the gradient of a target-row subset ---------------------------------------------------
    def target_backward(self, targets: "TargetRows") -> "TargetRowsBackward":
        """The target list's backward operator, cached ON the list (a cache on the
        partition keyed by id() kept every list that ever reached backward -- and its device
        operator and chunk buffers -- alive; now they go with the list)."""
        op = getattr(targets, "_backward_op", None)
        if op is None or op.part is not self:
            op = TargetRowsBackward(self, targets)
            targets._backward_op = op
        return op


def local_targets(idx: np.ndarray, start: int, stop: int):
    """Positions and local row ids of the targets that fall in [start, stop), original order."""
    idx = np.asarray(idx)
    pos = np.nonzero((idx >= start) & (idx < stop))[0]
    return pos, (idx[pos] - start).astype(np.int32)


class TargetRows:
    """A target list (the reference's `target_indices`, mlpconv.py:94) over the row partition.
    Every rank holds the whole global list `idx` (drawn with replacement, tensormain.py:226) and
    keeps the targets in its rows, in original order: `pos` (their places in the global list) and
    `rows` (a RowSelection of local row ids) -- every kept target (duplicates included) or, with
    distinct=True, the distinct rows only (increasing; `counts` their multiplicities). Every
    rank's distinct target ids are derived from the global list too (`block_distinct`): the
    backward operator is built without communication."""

    def __init__(self, idx, part: RowPartitionedCSR, distinct: bool = False):
        from .sparse import RowSelection
        idx = np.asarray(idx)
        self.idx = idx
        self.total = int(idx.size)
        self.pos, loc = local_targets(idx, part.start, part.stop)
        uniq, first, inverse, counts = np.unique(loc, return_index=True, return_inverse=True,
                                                 return_counts=True)
        self.first, self.inverse_host, self.counts = first, inverse, counts
        self.distinct = bool(distinct)
        dev = part.device
        self.rows = RowSelection((uniq if distinct else loc).astype(np.int32), dev)
        b = part.bounds
        self.block_distinct = [np.unique(idx[(idx >= b[q]) & (idx < b[q + 1])]).astype(np.int64)
                               for q in range(part.world)]

    def __len__(self):
        return int(self.pos.size)


class TargetRowsBackward:
    """The gradient of Y_p = (H_p . Z)[targets_p] with respect to the row-partitioned Z,
    exchanging only the targets' gradient rows (round 4).

    dZ = H[T]^T . g over the global target list T. With H symmetric, rank q's rows of it are
    H_q[:, D] . g_D: H_q with every column that is not a target dropped, times the gradient rows
    of the distinct targets D (duplicates summed first, in target order -- Theano's
    inc_subtensor, mlpconv.py:94). Each rank contributes its distinct targets' rows (its block of
    the exchange layout, padded to the largest count); the operator's kept columns are remapped
    into that layout. The single-GPU form is DeviceCSR.rows_transpose; against the round-3 form
    (scatter g into an N_p x C zero matrix, exchange it whole, multiply by all of H_q) the
    dropped terms are exact zeros, so the result is bitwise the same, on |D| / N of the exchange
    bytes and the targets' share of the nonzeros."""

    def __init__(self, part: RowPartitionedCSR, targets: TargetRows):
        # the list itself is not kept: it holds this operator (target_backward's cache), and a
        # reference back would make a cycle that only the cyclic GC frees
        self.part = part
        counts = [int(d.size) for d in targets.block_distinct]
        pad = max(max(counts, default=0), 1)
        pos_of = np.full(part.n, -1, dtype=np.int64)
        for q, d in enumerate(targets.block_distinct):
            pos_of[d] = q * pad + np.arange(d.size)
        Hg = part.local_global
        p = pos_of[Hg.indices]
        keep = p >= 0
        row_of = np.repeat(np.arange(Hg.shape[0]), np.diff(Hg.indptr))
        kept = np.zeros(Hg.shape[0] + 1, dtype=np.int64)
        np.cumsum(np.bincount(row_of[keep], minlength=Hg.shape[0]), out=kept[1:])
        A = sps.csr_matrix((Hg.data[keep], p[keep].astype(np.int32), kept.astype(np.int32)),
                           shape=(Hg.shape[0], part.world * pad))
        self.host = A
        self.nnz = int(A.nnz)
        # the padded all-gather sends every rank's block at the LARGEST count: with the targets
        # bunched on a few ranks (train rows are the first 60 % of the nodes) the exact-count
        # mesh moves far less (Twitter-US, 2 ranks: 144k vs 27k rows into rank 0)
        mean = sum(counts) / max(len(counts), 1)
        method = "mesh" if part.exchange == "mesh" or max(counts) > 1.25 * mean else "allgather"
        self.layout = ExchangeLayout(method, part.rank, part.world, part.group, counts=counts,
                                     pad=pad, sources=targets.block_distinct)
        if part._on_device:
            from .sparse import DeviceCSR
            self.A = DeviceCSR.from_scipy(A, part.device)
        else:
            self.A = A
        # the kept targets' rows -> this rank's distinct rows (None: already distinct, in order)
        self.to_distinct = None
        if not targets.distinct and targets.rows.n:
            from .sparse import RowSelection
            self.to_distinct = RowSelection(targets.inverse_host.astype(np.int32), part.device)
        self._bufs = {}

    def exchange_bytes(self, K: int) -> int:
        return self.layout.bytes_in(K)

    def backward(self, g: torch.Tensor, ops, n_chunks="auto", **kw) -> torch.Tensor:
        """dZ_p [n_local, K] from g, the gradient of this rank's kept target rows [len, K]."""
        part = self.part
        K = g.shape[1]
        n_d = self.layout.n_own
        if self.to_distinct is not None:
            g = ops.scatter_rows(n_d, self.to_distinct, g)
        out = ops.empty(part.n_local, K, part.device)
        if part.world == 1:
            if n_d == 0:  # an empty target list: no gradient flows into Z
                out.zero_()
                return out
            spmm_into_ops(ops, self.A, g, out, **kw)
            return out
        c = part._n_chunks(n_chunks, K)
        bufs = self._bufs.get((K, c))
        if bufs is None:
            bufs = self._bufs[(K, c)] = _ChunkBuffers(self.layout, K, c, part.device)
        bufs.fill(g)
        return pipelined_product(lambda A, Z, o, **k: spmm_into_ops(ops, A, Z, o, **k), self.A,
                                 bufs, out, **kw)


def spmm_into_ops(ops, A, Z, out, bias=None, act=None, rows=None, gate=None, mode="auto", **kw):
    """ops.spmm_into with the pipeline's keyword set."""
    return ops.spmm_into(A, Z, out, bias=bias, act=act, rows=rows, gate=gate, mode=mode)


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
            self.A = DeviceCSR.from_scipy(sps.csr_matrix(H), self.device)
            self._spmm = spmm
        else:
            self.A = sps.csr_matrix(H)
            self._spmm = local_spmm

    @property
    def width(self) -> int:
        return self.c1 - self.c0

    def spmm(self, Z_cols: torch.Tensor, **kw) -> torch.Tensor:
        return self._spmm(self.A, Z_cols, **kw)
