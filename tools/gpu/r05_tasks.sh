#!/bin/bash
# Round 5: the ordered plans' default task size (128): SpMM tests, World blocks, the Twitter-US
# SpMMs and step, the headline bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05k2
mkdir -p $out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_spmm_gpu.py tests/test_partition_world_gpu.py tests/test_fullsize_gpu.py tests/test_config3_gpu.py > $out/tests.log 2>&1 || { grep -E 'Error|assert|FAILED|passed|failed' $out/tests.log | cut -c1-300 | tail -30; exit 1; }
tail -1 $out/tests.log
PARTS=1,4,8 MODES=ordered,ordered:512,fast timeout -k 10 400 python -u tools/exp_block_modes.py > $out/blocks.log 2>&1 || { tail -5 $out/blocks.log; exit 1; }
grep slowest $out/blocks.log
for i in 1 2; do
  timeout -k 10 200 python -u tools/exp_spmm_lib.py > $out/lib$i.log 2>&1 || { tail -5 $out/lib$i.log; exit 1; }
  grep '^{' $out/lib$i.log
done
timeout -k 10 240 python -u tools/bench_train.py --config twitter-us --order propagate_first --warmup 5 --steps 20 > $out/us_pf.log 2>&1 || { tail -5 $out/us_pf.log; exit 1; }
echo "us_pf $(grep -o '"ms_per_step": [0-9.]*' $out/us_pf.log)"
timeout -k 10 240 python -u tools/bench_train.py --config twitter-us --order reference --warmup 5 --steps 20 > $out/us_ref.log 2>&1 || { tail -5 $out/us_ref.log; exit 1; }
echo "us_ref $(grep -o '"ms_per_step": [0-9.]*' $out/us_ref.log)"
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-variants --no-train-step --no-dense > $out/bench.log 2>&1 || { tail -5 $out/bench.log; exit 1; }
tail -1 $out/bench.log | cut -c1-300
