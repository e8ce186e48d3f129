#!/bin/bash
# round 6: split3's residuals as scalar subtractions vs packed (v_pk_add_f32): dense tests, then
# the output layer's kernels and the weight gradients, previous head vs the tree's library
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/ss; mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_dense_gpu.py > $out/tests.log 2>&1 || { tail -20 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 500 python -u tools/exp_dense_ab.py tools/varlibs/libgcg_head.so graphconvgeo_amd/libgcg_spmm.so --rounds=3 > $out/ab.jsonl 2>&1 || exit 1
for lib in tools/varlibs/libgcg_head.so graphconvgeo_amd/libgcg_spmm.so tools/varlibs/libgcg_head.so graphconvgeo_amd/libgcg_spmm.so; do
  GCG_LIB=$PWD/$lib timeout -k 10 300 python -u tools/exp_tn_math.py --rounds 1 > $out/tmp.log 2>&1 || { tail -5 $out/tmp.log; exit 1; }
  grep bf16x6 $out/tmp.log | sed "s|^|$lib |" >> $out/tn.txt
done
