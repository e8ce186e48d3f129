#!/bin/bash
# Whole -m gpu suite, smoke(), then the default bench line (what the driver runs at round end).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/full
mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -q --tb=short --timeout 600 --timeout-method thread -m gpu tests > $out/tests.log 2>&1 || { grep -E 'Error|assert|FAILED|passed|failed' $out/tests.log | cut -c1-300 | tail -30; exit 1; }
tail -2 $out/tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 400 python -u bench.py > $out/bench.log 2>&1 || { tail -30 $out/bench.log; exit 1; }
grep '^{' $out/bench.log > $out/bench.json
cut -c1-600 $out/bench.json
