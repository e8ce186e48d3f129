"""The 'auto' mode policy of graphconvgeo_amd.sparse.spmm (host logic, no GPU): split rows
('fast') only when one row could outlast the launch, the plan-less bitwise 'rowwise' form on
large graphs without hub rows, the bitwise 'ordered' plan otherwise."""
import numpy as np

from graphconvgeo_amd import sparse as gs
from graphconvgeo_amd.synth import synthetic_graph


class _Shape:
    def __init__(self, indptr):
        self.indptr = np.asarray(indptr)
        self.n_rows = self.indptr.size - 1
        self.nnz = int(self.indptr[-1])

    def max_row_nnz(self):
        return int(np.diff(self.indptr).max()) if self.n_rows else 0


def test_auto_uniform_graph_runs_rowwise():
    H = synthetic_graph(100_000, 1_000_000, kind="uniform", seed=5)
    assert gs.resolve_auto(_Shape(H.indptr)) == "rowwise"


def test_auto_powerlaw_graph_runs_ordered_plan():
    H = synthetic_graph(100_000, 1_000_000, kind="powerlaw", seed=5)
    assert gs.resolve_auto(_Shape(H.indptr)) == "ordered"


def test_auto_small_graph_keeps_plan():
    assert gs.resolve_auto(_Shape(np.arange(0, 2 * 30_000 + 1, 2))) == "ordered"


def test_auto_one_giant_row_splits():
    indptr = np.concatenate([[0], np.arange(1, 70_001) + 10_000_000])
    assert gs.resolve_auto(_Shape(indptr)) == "fast"


def test_auto_long_rows_below_the_launch_stay_ordered():
    """A longest row of ~nnz/1000 (the W1 gradient's tail gather: 43,164 of 43.5M) runs the
    bitwise ordered plan (whole-workgroup rows); split only past nnz/AUTO_SPLIT_RATIO."""
    n = 100_000
    lens = np.full(n, 400, dtype=np.int64)
    lens[0] = 40_000  # 40k of ~40M nonzeros
    indptr = np.concatenate([[0], np.cumsum(lens)])
    assert gs.resolve_auto(_Shape(indptr)) == "ordered"
    lens[0] = int(indptr[-1]) // gs.AUTO_SPLIT_RATIO + 1000
    indptr = np.concatenate([[0], np.cumsum(lens)])
    assert gs.resolve_auto(_Shape(indptr)) == "fast"
