#!/bin/bash
# Round 5: non-temporal streams. NT GEMM: abtree/libs/libgcg_fnt.so (A loads / C stores default
# policy) vs libgcg_ntall.so (both non-temporal); fused layer: libgcg_base.so vs libgcg_fnt.so.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05nts
mkdir -p $out
L=$GRAFT_REPO_ROOT/abtree/libs
for i in 1 2; do
  for v in ${NTV:-fnt ntall}; do
    GCG_LIB=$L/libgcg_$v.so timeout -k 10 300 python -u tools/exp_gemm_bf16x6.py --cfgs 0 --rounds 1 --reps 10 --shapes 840000x300x930,840000x930x300,1400000x300x930,531000x930x300,450000x300x256,450000x256x300 > $out/nt_${v}$i.log 2>&1 || { tail -5 $out/nt_${v}$i.log; exit 1; }
    echo "nt $v$i"; python - $out/nt_${v}$i.log <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d = json.loads(l); print(d['shape'], d['TF[bf16x6[0]]'], d['TF[f32[0]]'])
PY
  done
done
