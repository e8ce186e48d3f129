#!/bin/bash
# Round 3: cooperative ordered long rows -- SpMM parity, then per-rank block timings and the
# headline SpMM alone.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r03
mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -q --tb=short --timeout 300 --timeout-method thread -m gpu \
  tests/test_spmm_gpu.py tests/test_properties.py tests/test_fullsize_gpu.py tests/test_rectify_zero_gpu.py > $out/coop_tests.log 2>&1 || { tail -30 $out/coop_tests.log; exit 1; }
tail -2 $out/coop_tests.log
timeout -k 10 300 python -u tools/exp_block_modes.py powerlaw > $out/block_modes_coop.log 2>&1 || { tail -20 $out/block_modes_coop.log; exit 1; }
grep slowest $out/block_modes_coop.log
timeout -k 10 300 python -u bench.py --no-variants --no-train-step --no-dense --no-cpu-baseline > $out/bench_spmm.log 2>&1 || { tail -20 $out/bench_spmm.log; exit 1; }
grep '^{' $out/bench_spmm.log | cut -c1-400
