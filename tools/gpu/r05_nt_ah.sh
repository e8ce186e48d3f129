#!/bin/bash
# Round 5: bf16x6 NT G = 3 register-A tile without (3) and with (9, the default) the weight planes read one slot ahead.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05ah
mkdir -p $out
timeout -k 10 400 python -u tools/exp_gemm_bf16x6.py --cfgs "${CFGS:-0;3;9}" --rounds 3 --shapes ${SHAPES:-840000x300x930,840000x930x300,450000x300x256,450000x256x300} > $out/nt.log 2>&1 || { tail -20 $out/nt.log; exit 1; }
grep '^{' $out/nt.log | cut -c1-900
