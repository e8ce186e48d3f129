#!/bin/bash
# Round 3: hub-row microbench (single-wave vs cooperative), the coop threshold sweep, and the
# row-partitioned fit against MLPCONV.fit (2 gloo ranks on the one GPU).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r03
mkdir -p $out
for c in -1 1024; do GCG_COOP_MIN=$c timeout -k 10 120 python -u tools/exp_hub_row.py > $out/hub_$c.log 2>&1 || { tail -5 $out/hub_$c.log; exit 1; }; grep coop_min $out/hub_$c.log; done
COOPS="1024 4096" bash tools/gpu/coop_sweep.sh || exit 1
timeout -k 10 400 python -u -m pytest -x -q --tb=short --timeout 300 --timeout-method thread -m gpu \
  tests/test_dist_train_gpu.py > $out/dist_tests.log 2>&1 || { tail -30 $out/dist_tests.log; exit 1; }
tail -2 $out/dist_tests.log
