#!/bin/bash
# Round 5: the fused output layer's epilogue batched over the row tiles (this tree) vs one tile
# at a time (abtree/libs/libgcg_base.so), alternating; then the dense GPU tests on this tree.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05e
mkdir -p $out
B=$GRAFT_REPO_ROOT/abtree/libs/libgcg_base.so
for i in 1 2; do
  timeout -k 10 200 python -u tools/exp_fused_one.py > $out/new$i.log 2>&1 || { tail -5 $out/new$i.log; exit 1; }
  echo "new$i"; grep '^{' $out/new$i.log | grep bf16x6 | cut -c1-200
  GCG_LIB=$B timeout -k 10 200 python -u tools/exp_fused_one.py > $out/base$i.log 2>&1 || { tail -5 $out/base$i.log; exit 1; }
  echo "base$i"; grep '^{' $out/base$i.log | grep bf16x6 | cut -c1-200
done
grep '^{' $out/new1.log | grep f32 | cut -c1-200
grep '^{' $out/base1.log | grep f32 | cut -c1-200
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_dense_gpu.py tests/test_bf16x6_numerics.py > $out/tests.log 2>&1 || { grep -E 'Error|assert|FAILED|passed|failed' $out/tests.log | cut -c1-300 | tail -30; exit 1; }
tail -1 $out/tests.log
