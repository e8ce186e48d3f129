#!/bin/bash
# L2->fabric bytes of the SpMM in the mode 'auto' resolves to (uniform graph: rowwise):
# kernel trace, FETCH_SIZE and WRITE_SIZE in separate rocprofv3 passes, then the summary.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/pmc_spmm_auto
mkdir -p $out
for kind in uniform powerlaw; do
  tag=${kind}
  timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $out/$tag/kt -o kt -- python3 tools/exp_spmm_one.py $kind auto > $out/$tag.kt.log 2>&1 || { tail -5 $out/$tag.kt.log; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/$tag/f -o f -- python3 tools/exp_spmm_one.py $kind auto > $out/$tag.f.log 2>&1 || { tail -5 $out/$tag.f.log; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/$tag/w -o w -- python3 tools/exp_spmm_one.py $kind auto > $out/$tag.w.log 2>&1 || { tail -5 $out/$tag.w.log; exit 1; }
  eff=$(grep '^done' $out/$tag.kt.log | awk '{print $3}')
  python3 tools/pmc_summary.py --fetch $out/$tag/f --write $out/$tag/w --kernel spmm_rows_kernel \
      --workload twitter-world-$kind-k300-$eff --bytes 51696800004 --out $out/pmc_twitter-world-$kind-k300-$eff.json || exit 1
  grep -h "spmm_rows_kernel" $(find $out/$tag/kt -name "*kernel_stats.csv") | cut -c1-200
done
