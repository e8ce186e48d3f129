#!/bin/bash
# Distributed GCN training on one GPU box: parity tests (2 gloo ranks on one MI355X), the
# single-rank step, and a 2-rank gloo rehearsal of tools/bench_train_dist.py.
set -o pipefail
out=gpurun_out/dist_train
mkdir -p $out
timeout -k 10 500 python -u -m pytest tests/test_dist_train_gpu.py tests/test_dense_gpu.py tests/test_mlpconv_gpu.py -x -v --timeout 300 --timeout-method thread > $out/pytest.log 2>&1 || { tail -40 $out/pytest.log; exit 1; }
tail -4 $out/pytest.log
timeout -k 10 300 python -u tools/bench_train_dist.py --config twitter-us > $out/n1.log 2>&1 || { tail -20 $out/n1.log; exit 1; }
grep '^{' $out/n1.log
timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 tools/bench_train_dist.py --config twitter-us --dist-backend gloo --steps 3 --warmup 1 > $out/n2_gloo.log 2>&1 || { tail -20 $out/n2_gloo.log; exit 1; }
grep '^{' $out/n2_gloo.log
