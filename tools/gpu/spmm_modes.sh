#!/bin/bash
# SpMM mode / task-size / gather-depth sweep (tools/exp_spmm_modes.py), one process per env.
set -o pipefail
export SWEEP="ordered:0,ordered:32,ordered:64,ordered:128,rowwise:0,ordered:0"
for v in "GCG_INFLIGHT=0" "GCG_UNROLL=16"; do
  echo "== $v"
  env $v timeout -k 10 200 python -u tools/exp_spmm_modes.py uniform,powerlaw 2>&1 | grep -E "ms=" || exit 1
done
