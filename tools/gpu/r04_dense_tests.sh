#!/bin/bash
# The dense-kernel GPU tests alone (tests/test_dense_gpu.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r04/dense_tests
mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -q --tb=short --timeout 300 --timeout-method thread -m gpu tests/test_dense_gpu.py > $out/tests.log 2>&1 || { grep -E 'Error|assert|FAILED|passed|failed' $out/tests.log | cut -c1-300 | tail -30; exit 1; }
tail -1 $out/tests.log
