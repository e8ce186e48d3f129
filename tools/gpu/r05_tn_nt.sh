#!/bin/bash
# Round 5: split-K TN GEMM (dW2) operand loads non-temporal (this tree) vs default
# (abtree/libs/libgcg_base.so): the kernel alone (bench dense_kernels shapes) and the World step.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05tn
mkdir -p $out
for i in 1 2; do
  for v in cur base; do
    if [ $v = base ]; then export GCG_LIB=$GRAFT_REPO_ROOT/abtree/libs/libgcg_base.so; else unset GCG_LIB; fi
    timeout -k 10 200 python -u -c "
import json, torch, bench
print(json.dumps({k: v for k, v in bench.dense_kernels_bench(10, torch.device('cuda:0')).items() if 'tn' in k}))" > $out/tn_$v$i.log 2>&1 || { tail -5 $out/tn_$v$i.log; exit 1; }
    echo "$v$i $(grep '^{' $out/tn_$v$i.log | cut -c1-200)"
  done
done
unset GCG_LIB
TESTS=tests/test_dense_gpu.py bash tools/gpu/r05_train_ab.sh
