#!/bin/bash
# Round-2 GPU check: new/changed parity tests first, then the whole -m gpu suite, then the
# default bench line; rocprofv3's counter list is saved to look for DRAM-side TCC counters.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r02
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -v --tb=short --timeout 300 --timeout-method thread -m gpu \
  tests/test_rectify_zero_gpu.py tests/test_abi_gpu.py tests/test_mlpconv_gpu.py \
  tests/test_layers_gpu.py tests/test_config3_gpu.py > $out/new_tests.log 2>&1 \
  || { grep -E 'Error|assert|FAILED|passed|failed' $out/new_tests.log | cut -c1-300 | tail -30; exit 1; }
tail -3 $out/new_tests.log
timeout -k 10 600 python -u -m pytest -x -q --tb=short --timeout 300 --timeout-method thread -m gpu tests \
  --deselect tests/test_config3_gpu.py > $out/all_tests.log 2>&1 || { grep -E 'Error|assert|FAILED|passed|failed' $out/all_tests.log | cut -c1-300 | tail -30; exit 1; }
tail -3 $out/all_tests.log
timeout -k 10 400 python -u bench.py > $out/bench.log 2>&1 || { tail -30 $out/bench.log; exit 1; }
grep '^{' $out/bench.log > $out/bench.json
cut -c1-3000 $out/bench.json
(cd /tmp && timeout -k 5 60 rocprofv3 -L > $GRAFT_REPO_ROOT/$out/counters.txt 2>&1) || true
