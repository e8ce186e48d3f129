# bench.py's default (Twitter-World) multi-rank path with 4 ranks on one GPU over gloo
set -o pipefail
out=gpurun_out/rehearse4
mkdir -p $out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 4 --steps 5 --warmup 2 --dist-backend gloo --exchange allgather > $out/gloo4.log 2>&1 || { tail -30 $out/gloo4.log; exit 1; }
grep '^{' $out/gloo4.log | cut -c1-900
