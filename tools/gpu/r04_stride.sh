#!/bin/bash
# Round 4: 256-B aligned rows for wide operands (sparse.row_stride) -- the whole -m gpu suite,
# then the World reference-order training step with the new and the round-3 strides and the
# bf16x6 / f32 NT GEMM, alternating.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/r04/stride
mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -q --tb=short --timeout 600 --timeout-method thread -m gpu tests > $out/tests.log 2>&1 || { grep -E 'Error|assert|FAILED|passed|failed' $out/tests.log | cut -c1-300 | tail -30; exit 1; }
tail -1 $out/tests.log
for r in 1 2; do
  for leg in "" "--legacy-stride" "--nt-math f32" "--legacy-stride --nt-math f32"; do
    timeout -k 10 400 python -u tools/bench_train.py --config twitter-world --steps 10 $leg >> $out/train_world.jsonl 2>> $out/train.err || { tail -20 $out/train.err; exit 1; }
    tail -1 $out/train_world.jsonl | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["legacy_stride"], r["nt_math"], r["ms_per_step"])'
  done
done
