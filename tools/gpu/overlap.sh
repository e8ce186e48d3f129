#!/bin/bash
set -o pipefail
out=gpurun_out/overlap
mkdir -p $out
timeout -k 10 300 python -u tools/exp_cumask.py > $out/overlap.log 2>&1 || { tail -20 $out/overlap.log; exit 1; }
grep -v amdgpu.ids $out/overlap.log
