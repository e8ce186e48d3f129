"""Host-side layout rule of the dense operands (sparse.row_stride / empty_dense's row stride):
16-B aligned rows whose gathered K floats span the fewest 128-B lines."""
import math
import os

import pytest

from graphconvgeo_amd.sparse import row_stride

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def lines(start: int, nbytes: int) -> int:
    return (start % 128 + nbytes + 127) // 128


@pytest.mark.parametrize("k", list(range(1, 2100, 7)) + [256, 300, 930, 1024, 1500])
def test_row_stride_is_aligned_and_line_minimal(k):
    ld = row_stride(k)
    if k > 512 and ld % 64 == 0:
        # wide rows: 256-B aligned rows when that pads at most 1/12 of the row (round 4)
        assert ld - k < 64 and 12 * (ld - k) <= k
        return
    assert ld >= k and ld % 4 == 0 and ld < k + 36
    row_b, best = 4 * k, -(-4 * k // 128)
    starts = {(r * 4 * ld) % 128 for r in range(128)}
    worst = max(lines(s, row_b) for s in starts)
    k4 = (k + 3) // 4 * 4
    if ld != k4:
        # padding beyond round4(k) only when it buys the minimal line count on every row
        assert worst == best
        if (4 * ld) % 128 == 0:
            # 128-B aligned rows only when no unaligned stride within +32 floats gets there
            for cand in range(k4, k4 + 32, 4):
                if (4 * cand) % 128:
                    assert max(lines(s, row_b) for s in {(r * 4 * cand) % 128
                                                         for r in range(128)}) > best
    # never worse than the plain round4(k) stride
    base = max(lines(s, row_b) for s in {(r * 4 * k4) % 128 for r in range(128)})
    assert worst <= base


def test_row_stride_known_values():
    assert row_stride(300) == 304   # 1216-B rows: 10 lines each (1200-B rows: 10.25 on average)
    assert row_stride(930) == 960   # wide rows: 256-B aligned (3728-B rows: 30.3 vs 28.2 ms)
    assert row_stride(256) == 256   # 128-B aligned rows stay as they are
    assert row_stride(1500) == 1536  # wide rows: 256-B aligned
    assert row_stride(600) == 640 and row_stride(1000) == 1024 and row_stride(704) == 704
    assert row_stride(513) == 516    # 256-B alignment would pad 1/8 of the row: line rule
    assert row_stride(129) == 132 and row_stride(258) == 260
    assert row_stride(500) == 512    # the reference's default hidden size (tensormain.py:82)
    assert math.gcd(4 * row_stride(300), 128) == 64


def test_package_sets_graph_branch_streams_before_hip_starts():
    """The HIP runtime reads DEBUG_HIP_FORCE_GRAPH_QUEUES once, when it initialises: importing
    the package (in a fresh interpreter, no HIP yet) sets the default of 8, and an explicit
    setting wins (profiles/r06/graph_queues_ab*.txt)."""
    import subprocess
    import sys
    code = "import os, graphconvgeo_amd; print(os.environ['DEBUG_HIP_FORCE_GRAPH_QUEUES'])"
    env = {k: v for k, v in os.environ.items() if k != "DEBUG_HIP_FORCE_GRAPH_QUEUES"}
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                         cwd=ROOT, check=True).stdout.strip()
    assert out == "8"
    env["DEBUG_HIP_FORCE_GRAPH_QUEUES"] = "2"
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                         cwd=ROOT, check=True).stdout.strip()
    assert out == "2"
