#!/bin/bash
# Round 3: split-K layout sweep (tools/exp_tn_layout.py) + its PMC bytes for the World dW2 shape.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r03
mkdir -p $out
timeout -k 10 300 python -u tools/exp_tn_layout.py > $out/tn_layout.log 2>&1 || { tail -10 $out/tn_layout.log; exit 1; }
cut -c1-700 $out/tn_layout.log
