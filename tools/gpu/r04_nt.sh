#!/bin/bash
# Round 4: the persistent NT GEMM -- bitwise tests, then the bench's dense kernels with the
# persistent kernel on / off (GCG_NT_PERSIST), alternating, same box.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r04/nt
mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -q --tb=short --timeout 300 --timeout-method thread -m gpu \
  tests/test_dense_gpu.py -k "gemm_nt or matmul" > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -2 $out/tests.log
timeout -k 10 300 python3 -u tools/exp_nt_persist.py > $out/persist.jsonl 2>&1 || { tail -20 $out/persist.jsonl; exit 1; }
grep '^{' $out/persist.jsonl
