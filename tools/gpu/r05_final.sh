#!/bin/bash
# Round 5 final: the whole -m gpu suite, smoke(), the default bench line (profiles kept), then
# the training steps' kernel stats (Twitter-US and World, both orders).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05z
mkdir -p $out/prof
timeout -k 10 900 python -u -m pytest -q --tb=short --maxfail=25 --timeout 600 --timeout-method thread -m gpu tests > $out/tests.log 2>&1
rc=$?
grep -E '^FAILED|^ERROR|passed|failed' $out/tests.log | cut -c1-300 | tail -40
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 500 python -u bench.py --profile-dir $out/prof > $out/bench.log 2>&1 || { tail -30 $out/bench.log; exit 1; }
grep '^{' $out/bench.log > $out/bench.json
cut -c1-300 $out/bench.json
exit $rc
