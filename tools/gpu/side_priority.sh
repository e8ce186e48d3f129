set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/prio; mkdir -p $out
for r in 1 2; do
for cfg in twitter-world twitter-us; do
for p in 0 -1; do
timeout -k 10 300 python -u tools/bench_train.py --config $cfg --side-priority $p --steps 10 > $out/tmp.log 2>&1 || { tail -5 $out/tmp.log; exit 1; }
grep '^{' $out/tmp.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['config'], r['side_priority'], r['ms_per_step'])" | tee -a $out/res.txt
done; done; done
