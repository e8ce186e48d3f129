#!/bin/bash
# round 6: the whole -m gpu suite, smoke(), the default bench line with its live profiles, then
# the World training step in MLPCONV's default order (auto -> propagate-first) and the reference
# order, each a JSON line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/${OUT:-r06s}
mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -q --tb=short --timeout 600 --timeout-method thread -m gpu tests > $out/tests.log 2>&1 || { grep -E 'Error|assert|FAILED|passed|failed' $out/tests.log | cut -c1-300 | tail -30; exit 1; }
tail -2 $out/tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 400 python -u bench.py --profile-dir $out > $out/bench.log 2> $out/bench.err || { tail -30 $out/bench.err; exit 1; }
grep '^{' $out/bench.log > $out/bench.json
for order in auto reference; do
timeout -k 10 300 python -u tools/bench_train.py --config twitter-world --order $order > $out/train_world_$order.log 2>&1 || { tail -20 $out/train_world_$order.log; exit 1; }
grep '^{' $out/train_world_$order.log | cut -c1-200
done
