#!/bin/bash
# Round 4: the fused output layer on the bf16 matrix cores -- dense tests, then the A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r04/fused6
mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -q --tb=short --timeout 300 --timeout-method thread -m gpu tests/test_dense_gpu.py > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 300 python -u tools/exp_fused_compose.py > $out/compose.jsonl 2> $out/compose.err || { tail -20 $out/compose.err; exit 1; }
cat $out/compose.jsonl
