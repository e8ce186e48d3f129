#!/bin/bash
# Round 5: SpMM output rows stored non-temporal (abtree/libs/libgcg_nty.so) vs default
# (libgcg_base.so): the headline launch on both World graphs and the Twitter-US step's SpMMs.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05nty
mkdir -p $out
L=$GRAFT_REPO_ROOT/abtree/libs
for i in 1 2; do
  for v in base nty; do
    GCG_LIB=$L/libgcg_$v.so timeout -k 10 200 python -u tools/exp_headline.py > $out/head_$v$i.log 2>&1 || { tail -5 $out/head_$v$i.log; exit 1; }
    echo "$v$i"; grep '^{' $out/head_$v$i.log | cut -c1-200
    GCG_LIB=$L/libgcg_$v.so timeout -k 10 200 python -u tools/exp_spmm_lib.py > $out/lib_$v$i.log 2>&1 || { tail -5 $out/lib_$v$i.log; exit 1; }
    grep '^{' $out/lib_$v$i.log | cut -c1-300
  done
done
