set -o pipefail
bash tools/gpu_check.sh || exit 1
mkdir -p gpurun_out/r1s4
timeout -k 10 400 python3 -u tools/bench_graph.py > gpurun_out/r1s4/bench_graph.log 2>&1 || { tail -20 gpurun_out/r1s4/bench_graph.log; exit 1; }
grep '^{' gpurun_out/r1s4/bench_graph.log | cut -c1-300
