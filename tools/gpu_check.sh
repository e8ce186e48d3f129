set -o pipefail
mkdir -p gpurun_out/r1s4
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r1s4/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r1s4/pytest_gpu.log; exit 1; }
tail -5 gpurun_out/r1s4/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r1s4/smoke.log 2>&1 || { cat gpurun_out/r1s4/smoke.log; exit 1; }
cat gpurun_out/r1s4/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/r1s4/bench.log 2>&1 || { tail -20 gpurun_out/r1s4/bench.log; exit 1; }
grep '^{' gpurun_out/r1s4/bench.log
