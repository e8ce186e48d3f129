"""BASELINE config 5 on one GPU: the Twitter-World graph row-partitioned P = 2, 4, 8 ways, every
rank run in ONE process as P sequential shards.

Each rank's local block (RowPartitionedCSR: its rows of H, columns remapped into the exchange's
operand layout) runs the product path exactly as a rank of `bench.py --gpus P` does --
`spmm_pipelined` over the auto column-chunk count, the chunk buffers, `sparse.spmm` in the whole
graph's mode -- on the operand its exchange would deliver (distributed.LOOPBACK writes each
chunk's remote rows from the whole dense matrix, by `layout.operand_ids()`). Every block's rows
must be bitwise the unpartitioned `ordered` product (mlpconv.py:73,90: S.dot(H, .)), for every
exchange layout: the padded all-gather / mesh layout and the halo remap. The target-row backward
(TargetRowsBackward, the gradient of `[target_indices]`, mlpconv.py:94) is checked the same way,
with the train targets on the first 60 % of the nodes so that the last ranks hold none.
"""
import numpy as np
import pytest
import torch

from graphconvgeo_amd import distributed as D
from graphconvgeo_amd import sparse as gs
from graphconvgeo_amd.dist_train import GPUOps
from graphconvgeo_amd.synth import CONFIGS, synthetic_graph

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def world(cuda):
    cfg = CONFIGS["twitter-world"]
    H = synthetic_graph(cfg.n_nodes, cfg.n_edges)
    K = cfg.hidden
    A = gs.DeviceCSR.from_scipy(H, cuda, symmetric=True)
    assert gs.resolve_auto(A) == "ordered"
    g = torch.Generator(device=cuda).manual_seed(17)
    Z = gs.empty_dense(H.shape[0], K, cuda).normal_(generator=g)
    Y = gs.spmm(A, Z, mode="ordered")
    # train targets drawn with replacement from the first 60 % of the nodes (tensormain.py:226)
    rng = np.random.default_rng(23)
    n_tr = int(0.6 * H.shape[0])
    train = rng.choice(n_tr, size=n_tr).astype(np.int32)
    G = torch.randn((train.size, K), generator=g, device=cuda)
    # the round-3 form of the target backward: scatter (duplicates in target order) into an
    # N x K zero matrix, multiply by all of H (H^T = H)
    g_full = GPUOps.scatter_rows(H.shape[0], gs.RowSelection(train, cuda), G)
    dZ = gs.spmm(A, g_full, mode="ordered")
    del A, G
    return H, K, Z, Y, train, g_full, dZ


def _loopback(src):
    """What the exchange delivers: every remote row of the chunk from the whole matrix."""
    def fill(layout, buf, c0, c1):
        ids = torch.as_tensor(layout.operand_ids(), device=buf.device)
        remote = ids >= 0
        own = torch.zeros_like(remote)
        own[layout.own_off:layout.own_off + layout.n_own] = True
        rows = torch.nonzero(remote & ~own).squeeze(1)
        buf[rows, :c1 - c0] = src[ids[rows], c0:c1]
        return None
    return fill


@pytest.mark.parametrize("P", [2, 4, 8])
def test_world_partition_blocks_bitwise(world, cuda, P):
    H, K, Z, Y, _train, _g, _dZ = world
    plan = D.PartitionPlan(H, P)
    chunks = {}  # exchange -> the chunk counts its ranks chose
    try:
        D.LOOPBACK = _loopback(Z)
        for exchange in ("allgather", "mesh", "halo"):
            for r in range(P):
                part = D.RowPartitionedCSR(H, r, P, cuda, exchange=exchange, plan=plan)
                mode = part.resolve_mode("auto")
                assert mode == "ordered"  # the whole graph's mode at every N
                chunks.setdefault(exchange, set()).add(part.choose_chunks(K))
                Zl = gs.empty_dense(part.local_block_rows, K, cuda)
                Zl[:part.n_local] = Z[part.start:part.stop]
                Yp = gs.empty_dense(part.n_local, K, cuda)
                part.spmm_pipelined(Zl, Yp, n_chunks="auto", mode=mode)
                assert torch.equal(Yp, Y[part.start:part.stop]), (exchange, r)
                if r == 0:  # the chunk buffers hold exactly the operand rows the layout names
                    ids = part.layout.operand_ids()
                    assert ids.size == part.operand_rows()
                    assert np.array_equal(ids[part.layout.own_off:
                                              part.layout.own_off + part.n_local],
                                          np.arange(part.start, part.stop))
                del part, Zl, Yp
            torch.cuda.empty_cache()
    finally:
        D.LOOPBACK = None
    # every rank of one exchange agrees (the exchanges may differ: rows_in(exchange) differs)
    assert all(len(c) == 1 for c in chunks.values()), chunks


@pytest.mark.parametrize("P", [2, 8])
def test_world_partition_target_backward_bitwise(world, cuda, P):
    """dZ_q = H_q[:, D] . g_D for every rank q (only the distinct targets' rows exchanged) is
    bitwise (H . scatter(g))[rows of q]; at P = 8 ranks 5-7 hold no targets (counts 0 in the
    exchange) yet still receive the others' rows."""
    H, K, _Z, _Y, train, g_full, dZ = world
    plan = D.PartitionPlan(H, P)
    empty = 0
    try:
        D.LOOPBACK = _loopback(g_full)
        for r in range(P):
            part = D.RowPartitionedCSR(H, r, P, cuda, exchange="allgather", plan=plan)
            tg = D.TargetRows(train, part, distinct=True)
            bwd = part.target_backward(tg)
            own = tg.block_distinct[r]
            empty += own.size == 0
            g_own = g_full[torch.as_tensor(own, device=cuda)].contiguous()
            got = bwd.backward(g_own, GPUOps, mode="ordered")
            assert torch.equal(got, dZ[part.start:part.stop]), r
            assert part.target_backward(tg) is bwd
            del part, tg, bwd, got
    finally:
        D.LOOPBACK = None
    assert P < 8 or empty >= 1
