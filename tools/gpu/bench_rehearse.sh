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
# 4 and 8 ranks (halo exchange: all_to_all_single with per-peer splits), World graph at N = 8
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 4 --config twitter-us --steps 5 --warmup 2 --dist-backend gloo --no-cpu-baseline > $out/gloo4.log 2>&1 || { tail -30 $out/gloo4.log; exit 1; }
grep '^{' $out/gloo4.log | cut -c1-600
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29535 bench.py --gpus 8 --steps 3 --warmup 1 --dist-backend gloo --no-cpu-baseline > $out/gloo8.log 2>&1 || { tail -30 $out/gloo8.log; exit 1; }
grep '^{' $out/gloo8.log | cut -c1-900
