#!/bin/bash
# round 6: trainer tests after the default-order change, then bench.py's N > 1 path rehearsed
# over gloo on the one GPU at 2, 4 and 8 ranks exactly as the driver launches it (no extra flags):
# the headline line first, chunks_ab and the xGMI fit in it.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/${OUT:-r06c}
mkdir -p $out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -x -q --tb=short --timeout 300 --timeout-method thread tests/test_mlpconv_gpu.py tests/test_nonsymmetric_gpu.py tests/test_dist_train_gpu.py tests/test_config3_gpu.py > $out/tests.log 2>&1 || { grep -E 'Error|assert|FAILED|passed|failed' $out/tests.log | cut -c1-300 | tail -30; exit 1; }
tail -1 $out/tests.log
for n in 2 4 8; do
cfg=twitter-us; [ $n = 8 ] && cfg=twitter-world
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29540 + n)) bench.py --gpus $n --config $cfg --steps 5 --warmup 2 --dist-backend gloo --no-cpu-baseline > $out/gloo$n.log 2>&1 || { tail -30 $out/gloo$n.log; exit 1; }
grep '^{' $out/gloo$n.log | cut -c1-300
done
