#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r04/fused
mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -q --tb=short --timeout 300 --timeout-method thread -m gpu tests/test_dense_gpu.py > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for r in 1 2; do
timeout -k 10 300 python -u bench.py --config geotext --steps 10 --no-variants --no-train-step --no-cpu-baseline --no-live-pmc > $out/bench$r.log 2>&1 || { tail -20 $out/bench$r.log; exit 1; }
grep '^{' $out/bench$r.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print({k: v["TFLOPs"] for k, v in r["dense_kernels"].items() if isinstance(v, dict)})'
done
