#!/bin/bash
# Row-stride experiment: headline SpMM with Z/Y rows at ld = 300 (1200 B), 304 (1216 B: every
# row starts 0 or 64 B into a 128-B line, so it always spans exactly 10 lines) and 320 (1280 B,
# 128-B aligned rows), power-law and uniform degrees.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/ld_sweep
mkdir -p $out
for g in uniform powerlaw; do for ld in 0 304 320 0 304; do
timeout -k 10 300 python -u bench.py --graph $g --ld $ld --no-variants --no-train-step --no-dense --no-cpu-baseline > $out/${g}_${ld}.log 2>&1 || { tail -20 $out/${g}_${ld}.log; exit 1; }
python3 -c "import json; r=json.loads([l for l in open('$out/${g}_${ld}.log') if l.startswith('{')][0]); print('$g', $ld, r['ms_per_step'], r['roofline']['kernel_ms'], r['value'])"
done; done
