mkdir -p gpurun_out/d4
timeout -k 10 400 python -u -m pytest tests/test_dense_gpu.py tests/test_mlpconv_gpu.py tests/test_layers_gpu.py tests/test_pipeline_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/d4/pytest.log 2>&1; rc=$?; tail -5 gpurun_out/d4/pytest.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for cfg in twitter-us twitter-world; do for order in reference propagate_first; do
timeout -k 10 300 python -u tools/bench_train.py --config $cfg --order $order > gpurun_out/d4/train_${cfg}_${order}.log 2>&1 || exit 1
grep '^{' gpurun_out/d4/train_${cfg}_${order}.log
done; done
