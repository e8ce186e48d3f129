#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/gemm_nt
mkdir -p $out
timeout -k 10 500 python -u tools/exp_gemm_nt.py > $out/exp.log 2>&1 || { tail -20 $out/exp.log; exit 1; }
cat $out/exp.log | grep '^{'
