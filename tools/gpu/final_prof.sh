set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/fp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fp/sg -o run -- python3 -u tools/bench_graph.py --configs twitter-world --ops spgemm --spgemm-cpu-rows 20000 > gpurun_out/fp/sg.log 2>&1 || { tail -20 gpurun_out/fp/sg.log; exit 1; }
grep '^{' gpurun_out/fp/sg.log | cut -c1-250
for cfg in twitter-us twitter-world; do for order in reference propagate_first; do
timeout -k 10 300 python -u tools/bench_train.py --config $cfg --order $order > gpurun_out/fp/train_${cfg}_${order}.log 2>&1 || { tail -20 gpurun_out/fp/train_${cfg}_${order}.log; exit 1; }
grep '^{' gpurun_out/fp/train_${cfg}_${order}.log | cut -c1-300
done; done
