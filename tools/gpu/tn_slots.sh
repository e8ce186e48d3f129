#!/bin/bash
# round 6: gemm_tn6 split counts (GCG_TN6_SLOTS variant libraries) at the training step's shapes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/tns; mkdir -p $out
for lib in graphconvgeo_amd/libgcg_spmm.so tools/varlibs/libgcg_s4096.so tools/varlibs/libgcg_s16384.so tools/varlibs/libgcg_s32768.so; do
  GCG_LIB=$PWD/$lib timeout -k 10 300 python -u tools/exp_tn_math.py --rounds 1 > $out/tmp.log 2>&1 || { tail -5 $out/tmp.log; exit 1; }
  grep bf16x6 $out/tmp.log | sed "s|^|$lib |" >> $out/res.txt
done
