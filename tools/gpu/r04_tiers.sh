#!/bin/bash
# Round 4 experiment: three-tier gather hint (warm tier with an explicit load policy) -- parity
# tests, then the A/B on World power-law / US / World uniform. Needs commit 1259152 (knobs reverted).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/r04/tiers
mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -q --tb=short --timeout 200 --timeout-method thread -m gpu \
  tests/test_spmm_gpu.py -k "hint" > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 700 python -u tools/exp_hint_tiers.py > $out/tiers.jsonl 2> $out/tiers.err || { tail -20 $out/tiers.err; exit 1; }
python3 -c '
import json
for l in open("gpurun_out/r04/tiers/tiers.jsonl"):
    r = json.loads(l); print(r["graph"], r["hot_rows"], r["warm_rows"], r["ms_min"])'
