#!/bin/bash
# round 6: the weight gradients (dense.TN_MATH) f32 vs bf16x6 inside the training step, World
# and Twitter-US, alternated (the X-head GEMM f32 either way)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/tm; mkdir -p $out
for r in 1 2; do for cfg in twitter-world twitter-us; do for m in bf16x6 f32; do
timeout -k 10 300 python -u tools/bench_train.py --config $cfg --tn-math $m > $out/tmp.log 2>&1 || { tail -5 $out/tmp.log; exit 1; }
grep '^{' $out/tmp.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['config'], r['tn_math'], r['ms_per_step'])" >> $out/res.txt
done; done; done
cat $out/res.txt
