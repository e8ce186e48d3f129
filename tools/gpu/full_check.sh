#!/bin/bash
# All GPU tests, smoke, the dense-kernel bench and the four train-step benches.
set -o pipefail
out=gpurun_out/full
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1 || { tail -40 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 300 python -u tools/bench_dense.py --tiles occ2 > $out/bench_dense.log 2>&1 || { tail -20 $out/bench_dense.log; exit 1; }
grep -v '^{' $out/bench_dense.log | grep -v amdgpu.ids
for cfg in twitter-us twitter-world; do for order in reference propagate_first; do
timeout -k 10 300 python -u tools/bench_train.py --config $cfg --order $order > $out/train_${cfg}_${order}.log 2>&1 || { tail -20 $out/train_${cfg}_${order}.log; exit 1; }
grep '^{' $out/train_${cfg}_${order}.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['config'], r['order'], r['ms_per_step'])"
done; done
timeout -k 10 600 python -u bench.py > $out/bench.log 2>&1 || { tail -20 $out/bench.log; exit 1; }
grep '^{' $out/bench.log | cut -c1-700
timeout -k 10 600 python -u tools/bench_graph.py > $out/bench_graph.log 2>&1 || { tail -20 $out/bench_graph.log; exit 1; }
grep '^{' $out/bench_graph.log | cut -c1-400
bash tools/gpu/prof_spgemm.sh > $out/prof_spgemm.log 2>&1 || { tail -20 $out/prof_spgemm.log; exit 1; }
