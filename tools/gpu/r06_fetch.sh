#!/bin/bash
# round 6: library A/B of the fused layer's per-row reciprocal (tools/varlibs/*, GCG_LIB), then
# where its HBM reads come from: FETCH_SIZE and the L2 hit rate at 930 vs 64 classes
# (tools/exp_fused_fetch.py), one counter set per run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/${OUT:-r06f}
mkdir -p $out
if [ -n "$LIBS" ]; then
  timeout -k 10 600 python -u tools/exp_dense_ab.py graphconvgeo_amd/libgcg_spmm.so $LIBS --rounds=2 > $out/ab.jsonl 2> $out/ab.err || { tail -20 $out/ab.err; exit 1; }
  cat $out/ab.jsonl
fi
D=tools/exp_fused_fetch.py
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt -o kt -- python3 $D > $out/kt.log 2>&1 || { tail -5 $out/kt.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/f1 -o f1 -- python3 $D > $out/f1.log 2>&1 || { tail -5 $out/f1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $out/f2 -o f2 -- python3 $D > $out/f2.log 2>&1 || { tail -5 $out/f2.log; exit 1; }
find $out -name "*.csv" | head -20
