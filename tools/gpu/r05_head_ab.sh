#!/bin/bash
# Round 5: the W1 gradient's dense-head size (sparse.HYBRID_MAX_COLS) re-measured after the tail
# gather went ordered: propagate-first training steps, head 128 / 256 (default) / 512 columns.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05head
mkdir -p $out
run() {  # cols config log
  timeout -k 10 300 python -u -c "
import sys, runpy
import graphconvgeo_amd.sparse as gs
gs.HYBRID_MAX_COLS = $1
sys.argv = ['bench_train.py', '--config', '$2', '--order', 'propagate_first']
runpy.run_path('tools/bench_train.py', run_name='__main__')" > $3 2>&1 || { tail -5 $3; exit 1; }
  echo "head $1 $2 $(grep -o '"ms_per_step": [0-9.]*' $3)"
}
for cfg in twitter-us twitter-world; do
  for i in 1 2; do
    for c in 256 128 512; do
      run $c $cfg $out/${cfg}_$c$i.log || exit 1
    done
  done
done
