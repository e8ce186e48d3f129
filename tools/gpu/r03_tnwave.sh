#!/bin/bash
# Round 3: per-wave split-K tiles (tools/exp_tn_wave.py) for the World dW2 shape.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r03
mkdir -p $out
timeout -k 10 400 python -u tools/exp_tn_wave.py > $out/tn_wave.log 2>&1 || { tail -10 $out/tn_wave.log; exit 1; }
cut -c1-1500 $out/tn_wave.log
