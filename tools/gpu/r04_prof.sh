#!/bin/bash
# Round 4 evidence: (1) rocprofv3 kernel-trace stats of the bench command itself (headline only);
# (2) hash-stamped PMC summaries (FETCH_SIZE / WRITE_SIZE, separate passes) of the headline and
# uniform launches; (3) the N = 2 gloo rehearsal's step under a kernel trace at two step counts:
# copy kernels that scale with --steps would be staging copies inside the step.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
out=gpurun_out/r04/prof
mkdir -p $out
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/bench_kt -o bench -- python3 bench.py --no-variants --no-train-step --no-dense --no-cpu-baseline --no-live-pmc > $out/bench.log 2>&1 || { tail -30 $out/bench.log; exit 1; }
grep '^{' $out/bench.log > $out/bench.json
grep -h "spmm_rows_kernel" $(find $out/bench_kt -name "*kernel_stats.csv") | cut -c1-200
for kind in powerlaw uniform; do
  mode=ordered; [ $kind = uniform ] && mode=rowwise
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/pmc_${kind}_f -o f -- python3 tools/exp_spmm_one.py $kind $mode > $out/pmc_${kind}_f.log 2>&1 || { tail -5 $out/pmc_${kind}_f.log; exit 1; }
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/pmc_${kind}_w -o w -- python3 tools/exp_spmm_one.py $kind $mode > $out/pmc_${kind}_w.log 2>&1 || { tail -5 $out/pmc_${kind}_w.log; exit 1; }
  python3 tools/pmc_summary.py --fetch $out/pmc_${kind}_f --write $out/pmc_${kind}_w --workload twitter-world-$kind-k300-$mode --bytes 51696800004 --out $out/pmc_twitter-world-$kind-k300-$mode.json
done
for steps in 3 13; do
  port=$((29600 + steps))
  RANK=1 LOCAL_RANK=0 WORLD_SIZE=2 MASTER_ADDR=127.0.0.1 MASTER_PORT=$port timeout -k 10 300 python3 bench.py --gpus 2 --config twitter-us --dist-backend gloo --steps $steps --warmup 1 --no-alternatives > $out/n2_r1_$steps.log 2>&1 &
  r1=$!
  RANK=0 LOCAL_RANK=0 WORLD_SIZE=2 MASTER_ADDR=127.0.0.1 MASTER_PORT=$port timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/n2_kt_$steps -o n2 -- python3 bench.py --gpus 2 --config twitter-us --dist-backend gloo --steps $steps --warmup 1 --no-alternatives > $out/n2_r0_$steps.log 2>&1 || { tail -20 $out/n2_r0_$steps.log; kill $r1; exit 1; }
  wait $r1 || { tail -20 $out/n2_r1_$steps.log; exit 1; }
  echo "steps=$steps copy kernels:"; grep -h -i "copy\|Copy" $(find $out/n2_kt_$steps -name "*kernel_stats.csv") | cut -d, -f1,2 || echo "  none"
done
