#!/bin/bash
# Round 4: the histogram-sized gather hint and its capture guard, the masked tail with the
# per-call knob, then the headline on World and Twitter-US (hint sizes 32 / 15.5 MiB).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/r04
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --tb=short --timeout 300 --timeout-method thread -m gpu \
  tests/test_spmm_gpu.py -k "hint or tail or capture" > $out/hint_tests.log 2>&1 || { tail -40 $out/hint_tests.log; exit 1; }
tail -2 $out/hint_tests.log
for cfg in twitter-world twitter-us; do
  timeout -k 10 300 python -u bench.py --config $cfg --no-variants --no-dense --no-train-step --no-cpu-baseline > $out/hint_bench_$cfg.log 2>&1 || { tail -20 $out/hint_bench_$cfg.log; exit 1; }
  grep '^{' $out/hint_bench_$cfg.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["config"]["workload"], r["ms_per_step"], r["roofline"]["kernel_ms"], r["roofline"].get("frac"))'
done
python3 - <<'PY'
import torch, sys
sys.path.insert(0, ".")
from graphconvgeo_amd import sparse as gs
from graphconvgeo_amd.synth import CONFIGS, synthetic_graph
for name in ("twitter-world", "twitter-us"):
    cfg = CONFIGS[name]
    A = gs.DeviceCSR.from_scipy(synthetic_graph(cfg.n_nodes, cfg.n_edges), "cuda:0", symmetric=True)
    h = A.gather_hint(1216)
    print(name, "hot rows", A._hint_hot_rows, "MiB", round(A._hint_hot_rows * 1216 / 2**20, 1))
PY
