#!/bin/bash
# round 6: the HIP graph path against eager, with the HIP runtime's graph knobs
# (parallel-branch streams DEBUG_HIP_FORCE_GRAPH_QUEUES, packet capture
# DEBUG_CLR_GRAPH_PACKET_CAPTURE), Twitter-World and Twitter-US, alternated
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/gq; mkdir -p $out
run() {  # label, env..., -- args
  local label=$1; shift
  timeout -k 10 300 env "$@" > $out/tmp.log 2>&1 || { tail -5 $out/tmp.log; exit 1; }
  grep '^{' $out/tmp.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['config'], '$label', r['ms_per_step'])" >> $out/res.txt
}
for r in 1 2; do for cfg in twitter-world twitter-us; do
  run eager X=1 python -u tools/bench_train.py --config $cfg
  for q in ${QUEUES:-1 2 8}; do
    run graph_q$q DEBUG_HIP_FORCE_GRAPH_QUEUES=$q python -u tools/bench_train.py --config $cfg --graph
  done
  run graph X=1 python -u tools/bench_train.py --config $cfg --graph
  [ -n "$QUEUES" ] || run graph_nopkt DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 python -u tools/bench_train.py --config $cfg --graph
  [ -z "$HWQ" ] || run graph_q8_hw$HWQ DEBUG_HIP_FORCE_GRAPH_QUEUES=8 GPU_MAX_HW_QUEUES=$HWQ python -u tools/bench_train.py --config $cfg --graph
done; done
cat $out/res.txt
