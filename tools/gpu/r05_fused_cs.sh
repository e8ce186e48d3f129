#!/bin/bash
# Round 5: fused layer tiles (tile 3 = the 64-row tile with the cooperative A split) and the
# fused / dense GPU tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05cs
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --tb=short --timeout 300 --timeout-method thread -m gpu tests/test_dense_gpu.py > $out/tests.log 2>&1 || { grep -E 'Error|assert|FAILED|passed|failed' $out/tests.log | cut -c1-300 | tail -30; exit 1; }
tail -1 $out/tests.log
for i in 1 2; do
  timeout -k 10 200 python -u tools/exp_fused_one.py > $out/tiles$i.log 2>&1 || { tail -5 $out/tiles$i.log; exit 1; }
  grep '^{' $out/tiles$i.log | grep bf16x6 | cut -c1-160
done
