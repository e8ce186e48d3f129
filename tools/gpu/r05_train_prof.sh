#!/bin/bash
# Round 5: World training step (reference order, propagate-first): step time + kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05t
mkdir -p $out
export TMPDIR=/tmp
for o in reference propagate_first; do
  A="tools/bench_train.py --config twitter-world --order $o --warmup 3"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$o -o run -- python3 -u $A --steps 8 > $out/prof_$o.log 2>&1 || { tail -5 $out/prof_$o.log; exit 1; }
  find /tmp/prof_$o -name "*kernel_stats.csv" -exec cp {} $out/stats_$o.csv \;
  find /tmp/prof_$o -name "*kernel_trace.csv" -exec cp {} $out/trace_$o.csv \;
  echo "$o $(grep -o '"ms_per_step": [0-9.]*' $out/prof_$o.log)"
done
