#!/bin/bash
# Column-sum workgroup change (256-thread workgroups) and the row-batched rectify backward: its tests, then the World reference-order
# and propagate-first steps with kernel stats (compare profiles/r04/train/).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/r04/colsum
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --tb=short --timeout 120 --timeout-method thread -m gpu tests/test_relu_backward_gpu.py tests/test_rectify_zero_gpu.py tests/test_layers_gpu.py tests/test_mlpconv_gpu.py > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 120 python -u tools/exp_relu_bwd.py > $out/relu_bwd.log 2>&1 && cat $out/relu_bwd.log
GCG_RELU_ONE_ROW=1 timeout -k 10 120 python -u tools/exp_relu_bwd.py > $out/relu_bwd_one_row.log 2>&1 && cat $out/relu_bwd_one_row.log
for order in reference propagate_first; do
tag=twitter-world_${order}
timeout -k 10 300 python -u tools/bench_train.py --config twitter-world --order $order > $out/$tag.json.log 2>&1 || { tail -20 $out/$tag.json.log; exit 1; }
grep '^{' $out/$tag.json.log | cut -c1-120
done
tag=twitter-world_propagate_first_one_row
GCG_RELU_ONE_ROW=1 timeout -k 10 300 python -u tools/bench_train.py --config twitter-world --order propagate_first > $out/$tag.json.log 2>&1 || { tail -20 $out/$tag.json.log; exit 1; }
grep '^{' $out/$tag.json.log | cut -c1-120
tag=twitter-world_reference
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/$tag -o $tag -- python3 tools/bench_train.py --config twitter-world --order reference --steps 5 --warmup 2 > $out/$tag.prof.log 2>&1 || { tail -20 $out/$tag.prof.log; exit 1; }
find $out/$tag -name '*kernel_stats.csv' | head -1 | xargs grep -h "column_sum\|relu_backward" | cut -c1-40,80-200
