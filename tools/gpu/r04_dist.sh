#!/bin/bash
# Round 4: the partitioned path on the one GPU -- mesh / in-place all-gather / target-row
# backward tests (2 ranks over gloo), the per-phase step tool, bench --partitioned at world 1.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
out=gpurun_out/r04
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --tb=short --timeout 500 --timeout-method thread -m gpu \
  tests/test_dist_train_gpu.py tests/test_bench_gpu.py -k "two_ranks or row_partitioned" > $out/dist_tests.log 2>&1 || { tail -40 $out/dist_tests.log; exit 1; }
tail -3 $out/dist_tests.log
for order in propagate_first reference; do
  timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
    tools/bench_train_dist.py --config twitter-us --dist-backend gloo --order $order --phases --steps 4 --warmup 2 > $out/train_dist_$order.log 2>&1 || { tail -30 $out/train_dist_$order.log; exit 1; }
  grep '^{' $out/train_dist_$order.log
done
timeout -k 10 300 python -u bench.py --partitioned --no-cpu-baseline > $out/bench_part1.log 2>&1 || { tail -30 $out/bench_part1.log; exit 1; }
grep '^{' $out/bench_part1.log | cut -c1-400
timeout -k 10 300 python -u bench.py --no-variants --no-dense --no-train-step --no-cpu-baseline --no-live-pmc > $out/bench_plain.log 2>&1 || { tail -30 $out/bench_plain.log; exit 1; }
grep '^{' $out/bench_plain.log | cut -c1-300
