#!/bin/bash
# Round 5: HIP-graph replay vs eager on the Twitter-US propagate-first step, with the runtime's
# default kernel-argument placement and with HIP_FORCE_DEV_KERNARG=1 (kernargs in device memory).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05gk
mkdir -p $out
for i in 1 2; do
  for kv in 0 1; do
    for g in "" "--graph"; do
      HIP_FORCE_DEV_KERNARG=$kv timeout -k 10 200 python -u tools/bench_train.py --config twitter-us --order propagate_first $g > $out/k${kv}${g:+_graph}_$i.log 2>&1 || { tail -5 $out/k${kv}${g:+_graph}_$i.log; exit 1; }
      echo "kernarg=$kv ${g:-eager} $(grep -o '"ms_per_step": [0-9.]*' $out/k${kv}${g:+_graph}_$i.log)"
    done
  done
done
