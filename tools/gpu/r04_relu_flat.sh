#!/bin/bash
# Flat-access rectify backward (relu_backward_flat_kernel) vs the per-row mapping
# (GCG_RELU_ROW_MAPPING=1): tests, standalone kernel times, US / World propagate-first steps.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/r04/relu_flat
mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -q --tb=short --timeout 200 --timeout-method thread -m gpu tests/test_relu_backward_gpu.py tests/test_rectify_zero_gpu.py tests/test_layers_gpu.py tests/test_mlpconv_gpu.py tests/test_config3_gpu.py > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 120 python -u tools/exp_relu_bwd.py > $out/flat.log 2>&1 && cat $out/flat.log || exit 1
GCG_RELU_ROW_MAPPING=1 timeout -k 10 120 python -u tools/exp_relu_bwd.py > $out/row.log 2>&1 && cat $out/row.log || exit 1
for cfg in twitter-us twitter-world; do
for v in flat row flat2; do
  env=""; [ $v = row ] && env="GCG_RELU_ROW_MAPPING=1"
  env $env timeout -k 10 300 python -u tools/bench_train.py --config $cfg --order propagate_first > $out/${cfg}_$v.json.log 2>&1 || { tail -20 $out/${cfg}_$v.json.log; exit 1; }
  echo "$cfg $v $(grep '^{' $out/${cfg}_$v.json.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
done; done
