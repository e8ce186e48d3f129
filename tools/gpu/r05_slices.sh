#!/bin/bash
# Round 5: column-sliced hub rows -- bitwise tests, the A/B driver, P = 1/4/8 block timings,
# the headline bench (no CPU baseline).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05s
mkdir -p $out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_spmm_gpu.py tests/test_partition_world_gpu.py > $out/tests.log 2>&1 || { grep -E 'Error|assert|FAILED|passed|failed' $out/tests.log | cut -c1-300 | tail -30; exit 1; }
tail -1 $out/tests.log
timeout -k 10 300 python -u tools/exp_hub_slices.py > $out/slices.log 2>&1 || { tail -5 $out/slices.log; exit 1; }
cat $out/slices.log
PARTS=1,4,8 MODES=ordered,fast timeout -k 10 300 python -u tools/exp_block_modes.py > $out/blocks.log 2>&1 || { tail -5 $out/blocks.log; exit 1; }
grep slowest $out/blocks.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-variants --no-train-step --no-dense > $out/bench.log 2>&1 || { tail -5 $out/bench.log; exit 1; }
tail -1 $out/bench.log | cut -c1-400
