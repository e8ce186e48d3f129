#!/bin/bash
# Train-step evidence (BASELINE config 3 and the Twitter-World step): bench_train.py JSON lines
# plus rocprofv3 kernel-trace stats of the same command, both layer-2 orders.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/train_prof
mkdir -p $out
for cfg in twitter-us twitter-world; do for order in reference propagate_first; do
tag=${cfg}_${order}
timeout -k 10 300 python -u tools/bench_train.py --config $cfg --order $order > $out/$tag.json.log 2>&1 || { tail -20 $out/$tag.json.log; exit 1; }
grep '^{' $out/$tag.json.log | cut -c1-160
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/$tag -o $tag -- python3 tools/bench_train.py --config $cfg --order $order --steps 5 --warmup 2 > $out/$tag.prof.log 2>&1 || { tail -20 $out/$tag.prof.log; exit 1; }
done; done
