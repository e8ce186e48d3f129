set -o pipefail
mkdir -p gpurun_out/sg3
timeout -k 10 300 python -u -m pytest tests/test_spgemm_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/sg3/pytest.log 2>&1 || { tail -30 gpurun_out/sg3/pytest.log; exit 1; }
tail -2 gpurun_out/sg3/pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sg3/p -o run -- python3 -u tools/bench_graph.py --ops spgemm --spgemm-cpu-rows 20000 > gpurun_out/sg3/bench.log 2>&1 || { tail -20 gpurun_out/sg3/bench.log; exit 1; }
grep '^{' gpurun_out/sg3/bench.log | cut -c1-330
f=$(find gpurun_out/sg3/p -name "*kernel_stats.csv" | head -1); head -5 "$f" | cut -c1-60,200-300
