#!/bin/bash
# Round 5: GPU tests of the dense / trainer paths at this tree, then the Twitter-World training
# step (both orders) with this tree's library vs abtree/libs/libgcg_base.so, alternating.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05tab
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --tb=short --timeout 300 --timeout-method thread -m gpu ${TESTS:-tests/test_dense_gpu.py} tests/test_mlpconv_gpu.py tests/test_config3_gpu.py tests/test_layers_gpu.py tests/test_bf16x6_numerics.py > $out/tests.log 2>&1 || { grep -E 'Error|assert|FAILED|passed|failed' $out/tests.log | cut -c1-300 | tail -30; exit 1; }
tail -1 $out/tests.log
for i in 1 2; do
  for order in reference propagate_first; do
    timeout -k 10 300 python -u tools/bench_train.py --config ${CFG:-twitter-world} --order $order > $out/cur_${order}$i.log 2>&1 || { tail -20 $out/cur_${order}$i.log; exit 1; }
    echo "cur $order $(grep '^{' $out/cur_${order}$i.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
    GCG_LIB=$GRAFT_REPO_ROOT/abtree/libs/libgcg_base.so timeout -k 10 300 python -u tools/bench_train.py --config ${CFG:-twitter-world} --order $order > $out/base_${order}$i.log 2>&1 || { tail -20 $out/base_${order}$i.log; exit 1; }
    echo "base $order $(grep '^{' $out/base_${order}$i.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
  done
done
