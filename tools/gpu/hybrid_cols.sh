#!/bin/bash
# round 6: the X^T.g dense-head width (sparse.HYBRID_MAX_COLS) inside the training step,
# Twitter-World and Twitter-US, alternated
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/hc; mkdir -p $out
for r in 1 2; do for cfg in twitter-world twitter-us; do for c in 256 128 384 512; do
timeout -k 10 300 python -u tools/bench_train.py --config $cfg --hybrid-max-cols $c > $out/tmp.log 2>&1 || { tail -5 $out/tmp.log; exit 1; }
grep '^{' $out/tmp.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['config'], r['hybrid_max_cols'], r['ms_per_step'])" >> $out/res.txt
done; done; done
cat $out/res.txt
