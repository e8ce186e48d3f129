#!/bin/bash
# Profile one bench.py workload on the GPU box: kernel-trace stats + separate PMC passes
# (FETCH_SIZE, WRITE_SIZE, TCC hit/miss), summarised into gpurun_out/prof_<tag>_<workload>/pmc_<workload>.json.
# usage: tools/profile_bench.sh <round-tag> <bench args...>   (run from the repo root)
# The workload name uses the effective mode: bench's default 'auto' resolves to 'ordered'
# on the World graphs, so pass --mode explicitly when profiling anything else.
set -o pipefail
tag=$1; shift
export TMPDIR=/tmp
cfg=$(python3 - "$@" <<'PY'
import sys, argparse
ap = argparse.ArgumentParser(); ap.add_argument("--config", default="twitter-world")
ap.add_argument("--graph", default="powerlaw"); ap.add_argument("--hidden", type=int, default=300)
ap.add_argument("--mode", default="ordered"); a, _ = ap.parse_known_args(sys.argv[1:])
print(f"{a.config}-{a.graph}-k{a.hidden}-{a.mode}")
PY
)
out=gpurun_out/prof_${tag}_${cfg}
mkdir -p $out
run() { timeout -k 10 400 rocprofv3 "$@" --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline $BENCH_ARGS; }
BENCH_ARGS="$*"
run --kernel-trace --stats -d $out/trace -o t > $out/trace.log 2>&1 || { tail -5 $out/trace.log; exit 1; }
run --pmc FETCH_SIZE -d $out/fetch -o f > $out/fetch.log 2>&1 || { tail -5 $out/fetch.log; exit 1; }
run --pmc WRITE_SIZE -d $out/write -o w > $out/write.log 2>&1 || { tail -5 $out/write.log; exit 1; }
run --pmc TCC_HIT_sum TCC_MISS_sum -d $out/hits -o h > $out/hits.log 2>&1 || { tail -5 $out/hits.log; exit 1; }
bytes=$(grep -o '"algorithmic_bytes_per_launch": [0-9]*' $out/trace.log | head -1 | grep -o '[0-9]*$')
python3 tools/pmc_summary.py --fetch $out/fetch --write $out/write --hits $out/hits \
    --workload $cfg --bytes $bytes --out $out/pmc_${cfg}.json
cp $(find $out/trace -name '*kernel_stats.csv' | head -1) $out/${cfg}_kernel_stats.csv
grep '^{' $out/trace.log > $out/${cfg}_bench_under_rocprof.json || true
# gpurun merges only gpurun_out/ back; copy $out/{pmc_*.json,*_kernel_stats.csv} into profiles/ locally.
