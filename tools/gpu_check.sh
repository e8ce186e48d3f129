set -o pipefail
mkdir -p gpurun_out/r1s2
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r1s2/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r1s2/pytest_gpu.log; exit 1; }
tail -5 gpurun_out/r1s2/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r1s2/smoke.log 2>&1 || { cat gpurun_out/r1s2/smoke.log; exit 1; }
cat gpurun_out/r1s2/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/r1s2/bench.log 2>&1 || { tail -20 gpurun_out/r1s2/bench.log; exit 1; }
grep '^{' gpurun_out/r1s2/bench.log
