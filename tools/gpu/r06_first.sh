#!/bin/bash
# round 6, first GPU pass: the non-symmetric operator tests, trainer + bench contract tests,
# then the default bench line with its live profile
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r06a
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_nonsymmetric_gpu.py tests/test_mlpconv_gpu.py tests/test_dist_train_gpu.py \
  tests/test_bench_gpu.py > $OUT/tests.log 2>&1
timeout -k 10 400 python -u bench.py --profile-dir $OUT > $OUT/bench.log 2> $OUT/bench.err
