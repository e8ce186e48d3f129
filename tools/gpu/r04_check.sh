#!/bin/bash
# Round 4, first GPU pass: the masked-tail SpMM, the fused kernel's NaN-padding guard, the
# World full-size bench-layout test, the bench line with its live PMC pass.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/r04
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --tb=short --timeout 300 --timeout-method thread -m gpu \
  tests/test_spmm_gpu.py tests/test_dense_gpu.py tests/test_fullsize_gpu.py "$@" > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -3 $out/tests.log
timeout -k 10 400 python -u bench.py --no-train-step > $out/bench.log 2>&1 || { tail -30 $out/bench.log; exit 1; }
grep '^{' $out/bench.log > $out/bench.json
grep 'live PMC' $out/bench.log
python - <<'EOF'
import json
r = json.load(open("gpurun_out/r04/bench.json"))
print("value", r["value"], r["ms_per_step"], "roofline", {k: r["roofline"].get(k) for k in ("achieved", "frac", "edge_centric_frac", "traffic", "kernel_ms", "traffic_over_algorithmic")})
u = r["variants"]["uniform"]
print("uniform", u["kernel_ms"], {k: u["roofline"].get(k) for k in ("achieved", "frac", "edge_centric_frac", "traffic_over_algorithmic")})
print("k1500", r["variants"]["k1500"]["kernel_ms"], "fast", r["variants"]["fast"]["kernel_ms"])
print("cpu", r["cpu_baseline"])
EOF
