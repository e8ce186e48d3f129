#!/bin/bash
# Round 5: HIP-graph replay vs eager (Twitter-US propagate-first), graph batch sizes; the P = 8
# ordered blocks at task sizes 128 / 256 / 512.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05g
mkdir -p $out
run() {  # tag, env..., -- args
  local tag=$1; shift
  timeout -k 10 240 env "$@" > $out/train_$tag.log 2>&1 || { tail -5 $out/train_$tag.log; exit 1; }
  echo "$tag $(grep '^{' $out/train_$tag.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
}
A="python -u tools/bench_train.py --config twitter-us --order propagate_first --steps 20 --warmup 5"
run eager1 X=1 $A
run graph1 X=1 $A --graph
for b in 8 32 128 512; do run graph_b$b DEBUG_HIP_GRAPH_BATCH_SIZE=$b $A --graph; done
run eager2 X=1 $A
run graph2 X=1 $A --graph
PARTS=8 MODES=ordered:128,ordered:256,ordered,fast timeout -k 10 300 python -u tools/exp_block_modes.py > $out/blocks.log 2>&1 || { tail -5 $out/blocks.log; exit 1; }
grep slowest $out/blocks.log
