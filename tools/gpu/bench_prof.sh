#!/bin/bash
# rocprofv3 kernel-trace stats of the bench command itself (headline SpMM only: the extra
# measurements are switched off so spmm_rows_kernel's average is the headline launch's), for
# profiles/rNN/bench_kernel_stats.csv beside the JSON line printed under the profiler.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/bench_prof
mkdir -p $out
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt -o bench -- python3 bench.py --no-variants --no-train-step --no-dense --no-cpu-baseline > $out/bench.log 2>&1 || { tail -30 $out/bench.log; exit 1; }
grep '^{' $out/bench.log > $out/bench.json
find $out -name "*kernel_stats.csv"
