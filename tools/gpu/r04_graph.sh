#!/bin/bash
# Round 4: why the captured HIP graph of the training step replays slower
# than eager. Same Twitter-US propagate-first step: eager, eager without side streams, graph
# replay under the HIP runtime's graph-execution knobs (queues for parallel branches, packet
# capture), each in its own process.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r04/graph
mkdir -p $out
run() {  # name, env..., -- args
  local name=$1; shift
  timeout -k 10 200 env "$@" > $out/$name.log 2>&1 || { tail -20 $out/$name.log; exit 1; }
  echo "$name $(grep '^{' $out/$name.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["ms_per_step"])')"
}
B="python3 tools/bench_train.py --order propagate_first --steps 20 --warmup 5"
run eager GCG_X=1 $B
run eager_inline GCG_X=1 $B --inline-weight-grads --inline-head
run graph GCG_X=1 $B --graph
run graph_q1 DEBUG_HIP_FORCE_GRAPH_QUEUES=1 $B --graph
run graph_q2 DEBUG_HIP_FORCE_GRAPH_QUEUES=2 $B --graph
run graph_q4 DEBUG_HIP_FORCE_GRAPH_QUEUES=4 $B --graph
run graph_q8 DEBUG_HIP_FORCE_GRAPH_QUEUES=8 $B --graph
run graph_nopkt DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 $B --graph
run graph_inline GCG_X=1 $B --graph --inline-weight-grads --inline-head
run eager2 GCG_X=1 $B
run graph2 GCG_X=1 $B --graph
