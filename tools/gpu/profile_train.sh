#!/bin/bash
# Kernel-trace stats of the Twitter-World GCN train step (propagate-first order, fused MFMA
# output kernel) and of tools/bench_dense.py. Summaries land in gpurun_out/prof_train/.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/prof_train
mkdir -p $out
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $out/train -o t -- \
  python3 tools/bench_train.py --config twitter-world --order propagate_first --steps 4 --warmup 1 \
  > $out/train.log 2>&1 || { tail -5 $out/train.log; exit 1; }
cp $(find $out/train -name '*kernel_stats.csv' | head -1) $out/train_twitter-world_propagate_first_kernel_stats.csv
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/dense -o d -- \
  python3 tools/bench_dense.py --tiles rt4 --reps 5 > $out/dense.log 2>&1 || { tail -5 $out/dense.log; exit 1; }
cp $(find $out/dense -name '*kernel_stats.csv' | head -1) $out/dense_kernel_stats.csv
grep '^{' $out/train.log
