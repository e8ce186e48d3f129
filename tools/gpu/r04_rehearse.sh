#!/bin/bash
# Round 4: bench.py's multi-rank path rehearsed on one GPU over gloo (RCCL refuses several ranks
# on one device) with the round-4 pipeline -- copy-free step, auto chunks, exchange A/B
# (allgather / mesh / halo) -- Twitter-US at 2 and 4 ranks, Twitter-World at 2 and 8 ranks.
# Contract and code-path evidence only: gloo stages every exchange through host memory.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r04/rehearse
mkdir -p $out
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() {  # ranks config steps port
  timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node $1 --master-addr 127.0.0.1 --master-port $4 bench.py --gpus $1 --config $2 --steps $3 --warmup 1 --dist-backend gloo --no-cpu-baseline > $out/gloo$1_$2.log 2>&1 || { tail -30 $out/gloo$1_$2.log; exit 1; }
  grep '^{' $out/gloo$1_$2.log > $out/gloo$1_$2.json
  python3 -c "
import json; r=json.load(open('$out/gloo$1_$2.json')); d=r['distributed']; a=r.get('alternatives',{})
print($1, '$2', r['ms_per_step'], d['exchange'], d['chunks'], {k: v for k, v in a.items() if k.endswith('_ms')})"
}
run 2 twitter-us 3 29601
run 4 twitter-us 3 29602
run 2 twitter-world 2 29603
run 8 twitter-world 2 29604
