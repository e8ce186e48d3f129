#!/bin/bash
# SpMM HBM-side counters, power-law and uniform Twitter-World graphs, with and without
# non-temporal Y stores: FETCH_SIZE / WRITE_SIZE (separate passes) and the TCC->EA read
# requests split by destination (TCC_EA0_RDREQ_DRAM) plus the kernel-trace durations.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/pmc_spmm
mkdir -p $out
for kind in powerlaw uniform; do for nt in 0 1; do
  tag=${kind}_nt${nt}
  export GCG_SPMM_NT_STORE=$nt
  timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $out/$tag/kt -o kt -- python3 tools/exp_spmm_one.py $kind > $out/$tag.kt.log 2>&1 || { tail -5 $out/$tag.kt.log; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/$tag/f -o f -- python3 tools/exp_spmm_one.py $kind > $out/$tag.f.log 2>&1 || { tail -5 $out/$tag.f.log; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/$tag/w -o w -- python3 tools/exp_spmm_one.py $kind > $out/$tag.w.log 2>&1 || { tail -5 $out/$tag.w.log; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_32B_sum TCC_BUBBLE_sum --output-format csv -d $out/$tag/d -o d -- python3 tools/exp_spmm_one.py $kind > $out/$tag.d.log 2>&1 || { tail -5 $out/$tag.d.log; exit 1; }
  grep -h "spmm_rows_kernel" $(find $out/$tag/kt -name "*kernel_stats.csv") | cut -c1-200
done; done
