#!/bin/bash
set -o pipefail
out=gpurun_out/dense_check
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_dense_gpu.py tests/test_mlpconv_gpu.py tests/test_layers_gpu.py -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { tail -40 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
timeout -k 10 300 python -u tools/exp_gemm_bl.py > $out/bl.log 2>&1 || { tail -20 $out/bl.log; exit 1; }
grep -v amdgpu.ids $out/bl.log
