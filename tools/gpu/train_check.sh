#!/bin/bash
# After a trainer / epilogue change: the SpMM, dense, trainer and config-3 GPU tests, the
# epilogue-variant timings and the Twitter-US / World training-step benches.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/train_check
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --tb=short --timeout 300 --timeout-method thread -m gpu tests/test_spmm_gpu.py tests/test_dense_gpu.py tests/test_mlpconv_gpu.py tests/test_dist_train_gpu.py tests/test_config3_gpu.py tests/test_rectify_zero_gpu.py tests/test_layers_gpu.py > $out/tests.log 2>&1 || { grep -E 'Error|assert|FAILED|passed|failed' $out/tests.log | cut -c1-300 | tail -30; exit 1; }
tail -1 $out/tests.log
timeout -k 10 240 python -u tools/exp_epilogue.py twitter-us > $out/epi.log 2>&1 || { tail -20 $out/epi.log; exit 1; }
cat $out/epi.log
for cfg in twitter-us twitter-world; do
timeout -k 10 300 python -u tools/bench_train.py --config $cfg --order propagate_first > $out/train_${cfg}.log 2>&1 || { tail -20 $out/train_${cfg}.log; exit 1; }
grep '^{' $out/train_${cfg}.log | cut -c1-160
done
