#!/bin/bash
# Round 3: new gate / stream tests, then the one-GPU cost of the pipeline's SpMM split.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r03
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --tb=short --timeout 240 --timeout-method thread -m gpu \
  tests/test_rectify_zero_gpu.py tests/test_mlpconv_gpu.py tests/test_ops_gpu.py "$@" > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -3 $out/tests.log
timeout -k 10 300 python -u tools/exp_chunks.py > $out/chunks.log 2>&1 || { tail -20 $out/chunks.log; exit 1; }
cat $out/chunks.log
