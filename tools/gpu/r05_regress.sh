#!/bin/bash
# Previous commit's tree (abtree/) vs this tree: World blocks per mode (P = 1, 8), interleaved.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05r8
mkdir -p $out
for i in 1 2; do
  (cd abtree && PARTS=1,8 MODES=ordered,fast timeout -k 10 300 python -u tools/exp_block_modes.py) > $out/prev$i.log 2>&1 || { tail -5 $out/prev$i.log; exit 1; }
  echo "prev$i"; grep slowest $out/prev$i.log
  PARTS=1,8 MODES=ordered,fast timeout -k 10 300 python -u tools/exp_block_modes.py > $out/cur$i.log 2>&1 || { tail -5 $out/cur$i.log; exit 1; }
  echo "cur$i"; grep slowest $out/cur$i.log
done
