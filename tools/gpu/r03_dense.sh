#!/bin/bash
# Round 3: swizzled A chunk of the fused output layer -- dense parity, timing, PMC (LDS + MFMA).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r03
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --tb=short --timeout 240 --timeout-method thread -m gpu \
  tests/test_dense_gpu.py > $out/dense_tests.log 2>&1 || { tail -30 $out/dense_tests.log; exit 1; }
tail -1 $out/dense_tests.log
timeout -k 10 200 python -u tools/exp_fused_one.py > $out/fused_one.log 2>&1 || { tail -10 $out/fused_one.log; exit 1; }
cat $out/fused_one.log | cut -c1-300
OUT=$out/pmc_dense bash tools/gpu/pmc_nt.sh > /dev/null || exit 1
echo pmc done
