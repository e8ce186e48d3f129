#!/bin/bash
# Round 5: fused output layer, library A/B (abtree/libs/libgcg_$A.so vs libgcg_$B.so), alternating.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05fab
mkdir -p $out
for i in 1 2; do
  for v in ${A:-base} ${B:-nt}; do
    GCG_LIB=$GRAFT_REPO_ROOT/abtree/libs/libgcg_$v.so timeout -k 10 200 python -u tools/exp_fused_one.py > $out/${v}$i.log 2>&1 || { tail -5 $out/${v}$i.log; exit 1; }
    echo "$v$i"; grep '^{' $out/${v}$i.log | grep -E 'bf16x6.*"tile": 0|f32.*"tile": 0' | cut -c1-160
  done
done
