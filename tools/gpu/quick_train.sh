#!/bin/bash
# Dense kernel tests + the training-step benches (quick check after a dense-kernel change).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/quick_train
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --tb=short --timeout 300 --timeout-method thread -m gpu tests/test_dense_gpu.py tests/test_tmatmul_gpu.py tests/test_mlpconv_gpu.py tests/test_dist_train_gpu.py tests/test_config3_gpu.py > $out/tests.log 2>&1 || { grep -E 'Error|assert|FAILED|passed|failed' $out/tests.log | cut -c1-300 | tail -30; exit 1; }
tail -1 $out/tests.log
for cfg in twitter-us twitter-world; do for order in reference propagate_first; do
timeout -k 10 300 python -u tools/bench_train.py --config $cfg --order $order > $out/train_${cfg}_${order}.log 2>&1 || { tail -20 $out/train_${cfg}_${order}.log; exit 1; }
grep '^{' $out/train_${cfg}_${order}.log | cut -c1-120
done; done
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $out/bench.log 2>&1 || { tail -30 $out/bench.log; exit 1; }
grep '^{' $out/bench.log > $out/bench.json
python3 -c "import json; r=json.load(open('$out/bench.json')); print(json.dumps({k: r['train_step'][k] for k in ('reference','propagate_first','propagate_first_hip_graph')}))"
