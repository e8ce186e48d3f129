set -o pipefail
mkdir -p gpurun_out/sg2
timeout -k 10 400 python -u -m pytest tests/test_spgemm_gpu.py tests/test_graph_gpu.py tests/test_pipeline_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/sg2/pytest.log 2>&1 || { tail -30 gpurun_out/sg2/pytest.log; exit 1; }
tail -3 gpurun_out/sg2/pytest.log
timeout -k 10 400 python3 -u tools/exp_spgemm_alloc.py > gpurun_out/sg2/alloc.log 2>&1 || { tail -20 gpurun_out/sg2/alloc.log; exit 1; }
grep -v amdgpu.ids gpurun_out/sg2/alloc.log
timeout -k 10 400 python3 -u tools/bench_graph.py --ops spgemm > gpurun_out/sg2/bench_graph.log 2>&1 || { tail -20 gpurun_out/sg2/bench_graph.log; exit 1; }
grep '^{' gpurun_out/sg2/bench_graph.log
