#!/bin/bash
# Kernel trace of the Twitter-World GCN train step (propagate-first); stats + the per-dispatch
# trace land in gpurun_out/prof_train2/.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/prof_train2
mkdir -p $out
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $out/train -o t -- \
  python3 tools/bench_train.py --config twitter-world --order ${ORDER:-propagate_first} --steps 3 --warmup 1 \
  > $out/train.log 2>&1 || { tail -5 $out/train.log; exit 1; }
cp $(find $out/train -name '*kernel_stats.csv' | head -1) $out/stats.csv
cp $(find $out/train -name '*kernel_trace.csv' | head -1) $out/trace.csv
grep '^{' $out/train.log
