#!/bin/bash
# Round 5: the uniform World graph per SpMM mode / ordered task size (K = 300).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05un
mkdir -p $out
PARTS=1,8 MODES=rowwise,ordered,ordered:64,ordered:256,ordered:512,fast timeout -k 10 600 python -u tools/exp_block_modes.py uniform > $out/blocks.log 2>&1 || { tail -5 $out/blocks.log; exit 1; }
grep slowest $out/blocks.log
