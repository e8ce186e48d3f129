#!/bin/bash
# Round 5: dense GPU tests at this tree, then the NT tile A/B (G = 3 with / without planes ahead).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05d
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_dense_gpu.py tests/test_bf16x6_numerics.py tests/test_abi_gpu.py > $out/tests.log 2>&1 || { grep -E 'Error|assert|FAILED|passed|failed' $out/tests.log | cut -c1-300 | tail -30; exit 1; }
tail -1 $out/tests.log
SHAPES=840000x300x930,840000x930x300,1400000x300x930,531000x930x300 bash tools/gpu/r05_nt_ah.sh
