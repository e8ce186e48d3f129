#!/bin/bash
# Round 4: the N > 1 bench path (2 ranks over gloo on one GPU) after moving the exchange A/B
# into guarded functions, plus the bench tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
out=gpurun_out/r04/benchn2
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --tb=short --timeout 500 --timeout-method thread -m gpu tests/test_bench_gpu.py > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
