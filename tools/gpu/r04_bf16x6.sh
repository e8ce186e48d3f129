#!/bin/bash
# Round 4: NT GEMM on the bf16 matrix cores (bf16x6) vs the f32-MFMA kernel -- dense tests,
# then speed + error per tile on the output-layer shapes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r04/bf16x6
mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -q --tb=short --timeout 300 --timeout-method thread -m gpu tests/test_dense_gpu.py -k "nt" > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 500 python -u tools/exp_gemm_bf16x6.py ${BFX_ARGS:-} > $out/exp.jsonl 2> $out/exp.err || { tail -20 $out/exp.err; exit 1; }
cat $out/exp.jsonl
