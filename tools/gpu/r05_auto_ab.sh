#!/bin/bash
# Round 5: 'auto' split ratio nnz/512 (this tree) vs the round-2 nnz/2048: the World / US training
# steps alternating (the old ratio set in-process before tools/bench_train.py runs), then the
# whole -m gpu suite.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05auto
mkdir -p $out
run() {  # ratio config order log
  timeout -k 10 300 python -u -c "
import sys, runpy
import graphconvgeo_amd.sparse as gs
gs.AUTO_SPLIT_RATIO = $1
sys.argv = ['bench_train.py', '--config', '$2', '--order', '$3']
runpy.run_path('tools/bench_train.py', run_name='__main__')" > $4 2>&1 || { tail -5 $4; exit 1; }
  echo "ratio $1 $2 $3 $(grep -o '"ms_per_step": [0-9.]*' $4)"
}
for cfg in twitter-world twitter-us; do
  for i in 1 2; do
    for o in propagate_first reference; do
      run 512 $cfg $o $out/new_${cfg}_${o}$i.log || exit 1
      run 2048 $cfg $o $out/old_${cfg}_${o}$i.log || exit 1
    done
  done
done
timeout -k 10 1000 python -u -m pytest -q --tb=short --maxfail=10 --timeout 600 --timeout-method thread -m gpu tests > $out/tests.log 2>&1
grep -E '^FAILED|^ERROR|passed|failed' $out/tests.log | tail -12
