#!/bin/bash
# Round 3: split-K + fused output layer after the buffer-descriptor loads; dense GPU tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r03
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --tb=short --timeout 300 --timeout-method thread -m gpu tests/test_dense_gpu.py tests/test_mlpconv_gpu.py tests/test_config3_gpu.py tests/test_ops_gpu.py > $out/dense_tests.log 2>&1 || { grep -E 'Error|assert|FAILED|passed|failed' $out/dense_tests.log | cut -c1-300 | tail -30; exit 1; }
tail -2 $out/dense_tests.log
timeout -k 10 400 python -u tools/exp_tn_wave.py > $out/tn_wave3.log 2>&1 || { tail -10 $out/tn_wave3.log; exit 1; }
cut -c1-1500 $out/tn_wave3.log
timeout -k 10 300 python -u tools/exp_fused_one.py > $out/fused_one.log 2>&1 || { tail -10 $out/fused_one.log; exit 1; }
cut -c1-600 $out/fused_one.log
