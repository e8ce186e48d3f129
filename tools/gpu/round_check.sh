set -o pipefail
bash tools/gpu_check.sh || exit 1
mkdir -p gpurun_out/r1s4
timeout -k 10 400 python3 -u tools/bench_graph.py > gpurun_out/r1s4/bench_graph.log 2>&1 || { tail -20 gpurun_out/r1s4/bench_graph.log; exit 1; }
grep '^{' gpurun_out/r1s4/bench_graph.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r1s4/sg -o run -- python3 -u tools/bench_graph.py --configs twitter-world --ops spgemm --spgemm-cpu-rows 20000 > gpurun_out/r1s4/sg.log 2>&1 || { tail -20 gpurun_out/r1s4/sg.log; exit 1; }
grep '^{' gpurun_out/r1s4/sg.log | cut -c1-250
