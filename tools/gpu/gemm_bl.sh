#!/bin/bash
set -o pipefail
out=gpurun_out/gemm_bl
mkdir -p $out
timeout -k 10 300 python -u tools/exp_gemm_bl.py > $out/bl.log 2>&1 || { tail -20 $out/bl.log; exit 1; }
grep -v amdgpu.ids $out/bl.log
