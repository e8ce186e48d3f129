#!/bin/bash
# A/B: this tree's library vs a variant (abtree/libs/libgcg_u16.so: the U = 16 batch for the
# 128-nonzero ordered tasks) on the World blocks and the Twitter-US SpMMs; then the GPU tests
# of the ops / layers / trainer.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05u
mkdir -p $out
W=$GRAFT_REPO_ROOT/abtree/libs/libgcg_u16.so
for i in 1 2; do
  PARTS=1,8 MODES=ordered timeout -k 10 300 python -u tools/exp_block_modes.py > $out/cur$i.log 2>&1 || { tail -5 $out/cur$i.log; exit 1; }
  echo "cur$i"; grep slowest $out/cur$i.log
  GCG_LIB=$W PARTS=1,8 MODES=ordered timeout -k 10 300 python -u tools/exp_block_modes.py > $out/u16_$i.log 2>&1 || { tail -5 $out/u16_$i.log; exit 1; }
  echo "u16_$i"; grep slowest $out/u16_$i.log
done
timeout -k 10 200 python -u tools/exp_spmm_lib.py > $out/lib_cur.log 2>&1 || { tail -5 $out/lib_cur.log; exit 1; }
grep '^{' $out/lib_cur.log
GCG_LIB=$W timeout -k 10 200 python -u tools/exp_spmm_lib.py > $out/lib_u16.log 2>&1 || { tail -5 $out/lib_u16.log; exit 1; }
grep '^{' $out/lib_u16.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ops_gpu.py tests/test_layers_gpu.py tests/test_mlpconv_gpu.py > $out/tests.log 2>&1 || { grep -E 'Error|assert|FAILED|passed|failed' $out/tests.log | cut -c1-300 | tail -30; exit 1; }
tail -1 $out/tests.log
