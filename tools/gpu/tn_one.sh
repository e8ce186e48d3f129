#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/tn_one
mkdir -p $out
timeout -k 10 300 python -u tools/exp_tn_one.py > $out/exp.log 2>&1 || { tail -20 $out/exp.log; exit 1; }
grep '^{' $out/exp.log
timeout -k 10 300 python -u -m pytest -x -q --tb=short --timeout 300 --timeout-method thread -m gpu tests/test_dense_gpu.py > $out/tests.log 2>&1 || { grep -E 'Error|assert|FAILED|passed|failed' $out/tests.log | cut -c1-300 | tail -30; exit 1; }
tail -1 $out/tests.log
