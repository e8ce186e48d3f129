#!/bin/bash
# round 6: the graph tests and graph-vs-eager steps with the package's default graph streams
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/gd; mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_mlpconv_gpu.py -k "graph" > $out/tests.txt 2>&1 || { tail -20 $out/tests.txt; exit 1; }
tail -2 $out/tests.txt
for r in 1 2; do for cfg in twitter-world twitter-us; do for g in "" --graph; do
timeout -k 10 300 python -u tools/bench_train.py --config $cfg $g > $out/tmp.log 2>&1 || { tail -5 $out/tmp.log; exit 1; }
grep '^{' $out/tmp.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['config'], 'graph' if r['hip_graph'] else 'eager', r['ms_per_step'])" >> $out/res.txt
done; done; done
cat $out/res.txt
