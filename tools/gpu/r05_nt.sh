#!/bin/bash
# Round 5: bf16x6 NT tiles incl. the wide-column register-A forms (9: 256 x 320, 10: 128 x 320,
# 11: 256 x 256) on the output-layer shapes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05n
mkdir -p $out
timeout -k 10 300 python -u tools/exp_gemm_bf16x6.py --cfgs "0;3;9;10;11" --rounds 2 --shapes 531000x930x300,840000x930x300,1400000x300x930,450000x256x300,450000x300x256 > $out/nt.log 2>&1 || { tail -20 $out/nt.log; exit 1; }
grep '^{' $out/nt.log | cut -c1-600
