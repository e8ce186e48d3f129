set -o pipefail
bash tools/gpu/prof_spgemm.sh || exit 1
mkdir -p gpurun_out/graph
timeout -k 10 400 python3 -u tools/bench_graph.py > gpurun_out/graph/bench_graph.log 2>&1 || { tail -20 gpurun_out/graph/bench_graph.log; exit 1; }
grep '^{' gpurun_out/graph/bench_graph.log
