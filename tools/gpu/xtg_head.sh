#!/bin/bash
set -o pipefail
out=gpurun_out/xtg
mkdir -p $out
timeout -k 10 300 python -u tools/exp_xtg_head.py > $out/head.log 2>&1 || { tail -20 $out/head.log; exit 1; }
grep -v amdgpu.ids $out/head.log
