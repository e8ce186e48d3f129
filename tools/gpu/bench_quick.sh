#!/bin/bash
# Default bench line without the CPU baselines (quick check of the GPU fields).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/bench_quick
mkdir -p $out
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $out/bench.log 2>&1 || { tail -30 $out/bench.log; exit 1; }
grep '^{' $out/bench.log > $out/bench.json
python3 -c "import json; r=json.load(open('$out/bench.json')); print(r['value'], r['ms_per_step'], json.dumps(r['variants']))"
