#!/bin/bash
# SpMM epilogue-variant costs (US, World) + one Twitter-US propagate-first step timeline.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/epi
mkdir -p $out
for cfg in twitter-us twitter-world; do
timeout -k 10 240 python -u tools/exp_epilogue.py $cfg > $out/epi_$cfg.log 2>&1 || { tail -20 $out/epi_$cfg.log; exit 1; }
cat $out/epi_$cfg.log
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/us -o kt -- python3 tools/bench_train.py --config twitter-us --order propagate_first --steps 3 --warmup 1 > $out/us.log 2>&1 || { tail -20 $out/us.log; exit 1; }
python3 tools/step_timeline.py $out/us --steps 4 > $out/us.timeline.txt || exit 1
tail -70 $out/us.timeline.txt
