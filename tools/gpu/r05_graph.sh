#!/bin/bash
# Round 5: HIP-graph replay vs eager (Twitter-US propagate-first), main stream at default vs
# high priority (side streams at default).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05g4
mkdir -p $out
A="tools/bench_train.py --config twitter-us --order propagate_first --warmup 5 --steps 20"
run() {  # tag, env/args
  local tag=$1; shift
  timeout -k 10 240 env "$@" > $out/$tag.log 2>&1 || { tail -5 $out/$tag.log; exit 1; }
  echo "$tag $(grep -o '"ms_per_step": [0-9.]*' $out/$tag.log)"
}
for i in 1 2; do
  run eager$i X=1 python -u $A
  run graph$i X=1 python -u $A --graph
  run eager_prio$i X=1 python -u $A --main-priority
  run graph_prio$i X=1 python -u $A --graph --main-priority
done
