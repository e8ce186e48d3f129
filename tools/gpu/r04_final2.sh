#!/bin/bash
# Round 4 final evidence at the head: whole -m gpu suite, smoke(), the default bench line (with
# its live PMC pass), the bench under a kernel trace, and hash-stamped PMC summaries.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
out=gpurun_out/r04/final2
mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -q --tb=short --timeout 600 --timeout-method thread -m gpu tests > $out/tests.log 2>&1 || { grep -E 'Error|assert|FAILED|passed|failed' $out/tests.log | cut -c1-300 | tail -30; exit 1; }
tail -1 $out/tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 500 python -u bench.py > $out/bench.log 2>&1 || { tail -30 $out/bench.log; exit 1; }
grep '^{' $out/bench.log > $out/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/bench_kt -o bench -- python3 bench.py --no-variants --no-train-step --no-dense --no-cpu-baseline --no-live-pmc > $out/bench_prof.log 2>&1 || { tail -30 $out/bench_prof.log; exit 1; }
grep '^{' $out/bench_prof.log > $out/bench_under_rocprof.json
for kind in powerlaw uniform; do
  mode=ordered; [ $kind = uniform ] && mode=rowwise
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/pmc_${kind}_f -o f -- python3 tools/exp_spmm_one.py $kind $mode > $out/pmc_${kind}_f.log 2>&1 || { tail -5 $out/pmc_${kind}_f.log; exit 1; }
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/pmc_${kind}_w -o w -- python3 tools/exp_spmm_one.py $kind $mode > $out/pmc_${kind}_w.log 2>&1 || { tail -5 $out/pmc_${kind}_w.log; exit 1; }
  python3 tools/pmc_summary.py --fetch $out/pmc_${kind}_f --write $out/pmc_${kind}_w --workload twitter-world-$kind-k300-$mode --bytes 51696800004 --out $out/pmc_twitter-world-$kind-k300-$mode.json > /dev/null
done
python3 - <<'PY'
import json
r = json.load(open("gpurun_out/r04/final2/bench.json"))
rf = r["roofline"]
print("bench", r["value"], r["ms_per_step"], {k: rf.get(k) for k in ("achieved", "frac", "edge_centric_frac", "kernel_ms")})
print("uniform", r["variants"]["uniform"]["roofline"]["frac"], "dense", {k: v["TFLOPs"] for k, v in r["dense_kernels"].items() if isinstance(v, dict)})
print("train", {k: v["ms_per_step"] for k, v in r["train_step"].items() if isinstance(v, dict) and "ms_per_step" in v})
PY
