#!/bin/bash
set -o pipefail
out=gpurun_out/tn
mkdir -p $out
timeout -k 10 400 python -u tools/exp_tn_shapes.py > $out/tn.log 2>&1 || { tail -20 $out/tn.log; exit 1; }
grep -v amdgpu.ids $out/tn.log
