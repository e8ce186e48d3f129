cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sgprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sgprof/p -o run -- python3 -u tools/bench_graph.py --configs twitter-world --ops spgemm --spgemm-cpu-rows 1000 > gpurun_out/sgprof/out.log 2>&1
find gpurun_out/sgprof -name "*kernel_stats.csv" | head -3
f=$(find gpurun_out/sgprof -name "*kernel_stats.csv" | head -1); head -15 "$f" | cut -c1-220
