#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/timeline
mkdir -p $out
for cfg in twitter-us twitter-world; do
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/$cfg -o kt -- python3 tools/bench_train.py --config $cfg --order propagate_first --steps 3 --warmup 1 > $out/$cfg.log 2>&1 || { tail -20 $out/$cfg.log; exit 1; }
python3 tools/step_timeline.py $out/$cfg --steps 4 > $out/$cfg.timeline.txt || exit 1
tail -45 $out/$cfg.timeline.txt
done
