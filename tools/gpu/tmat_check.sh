#!/bin/bash
set -o pipefail
out=gpurun_out/tmat
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_relu_backward_gpu.py tests/test_tmatmul_gpu.py tests/test_dense_gpu.py tests/test_layers_gpu.py tests/test_mlpconv_gpu.py tests/test_dist_train_gpu.py -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { tail -40 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log


for cfg in twitter-us twitter-world; do for order in reference propagate_first; do
timeout -k 10 300 python -u tools/bench_train.py --config $cfg --order $order > $out/train_${cfg}_${order}.log 2>&1 || { tail -20 $out/train_${cfg}_${order}.log; exit 1; }
grep '^{' $out/train_${cfg}_${order}.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['config'], r['order'], r['ms_per_step'])"
done; done
