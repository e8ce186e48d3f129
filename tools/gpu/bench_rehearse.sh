#!/bin/bash
# bench.py's multi-rank path rehearsed on one GPU: 2 ranks over gloo (RCCL refuses two ranks
# on one device), plus the partitioned path at N = 1.
set -o pipefail
out=gpurun_out/rehearse
mkdir -p $out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u bench.py --config twitter-us --steps 5 --warmup 2 --partitioned --no-cpu-baseline > $out/part1.log 2>&1 || { tail -20 $out/part1.log; exit 1; }
grep '^{' $out/part1.log | cut -c1-400
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --config twitter-us --steps 5 --warmup 2 --dist-backend gloo --no-cpu-baseline > $out/gloo2.log 2>&1 || { tail -30 $out/gloo2.log; exit 1; }
grep '^{' $out/gloo2.log | cut -c1-600
