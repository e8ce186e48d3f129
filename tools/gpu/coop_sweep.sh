#!/bin/bash
# GCG_COOP_MIN sweep of the ordered-mode cooperative long rows (tools/exp_block_modes.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r03
mkdir -p $out
timeout -k 10 200 python -u -m pytest -x -q --tb=short --timeout 150 --timeout-method thread -m gpu \
  tests/test_spmm_gpu.py -k "cooperative or bitwise" > $out/coop_tests2.log 2>&1 || { tail -30 $out/coop_tests2.log; exit 1; }
tail -1 $out/coop_tests2.log
for c in -1 ${COOPS:-1024 2048 4096 8192}; do
  GCG_COOP_MIN=$c MODES=ordered timeout -k 10 200 python -u tools/exp_block_modes.py powerlaw > $out/coop_$c.log 2>&1 || { tail -5 $out/coop_$c.log; exit 1; }
  echo "coop_min=$c $(grep slowest $out/coop_$c.log | tr '\n' ' ')"
done
