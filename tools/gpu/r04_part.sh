#!/bin/bash
# Round 4: cost-aware row partition (slowest / mean block at P = 4, 8) and the masked-tail
# dwordx4 SpMM at C = 930 / 129 against the old dwordx2 / dword gathers (GCG_SPMM_NO_TAIL=1).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r04
mkdir -p $out
KS=129,132,930,932 GCG_SPMM_NO_TAIL=1 timeout -k 10 300 python -u tools/exp_spmm_k.py powerlaw,uniform > $out/spmm_k_notail.jsonl 2>&1 || { tail -20 $out/spmm_k_notail.jsonl; exit 1; }
KS=129,132,930,932 timeout -k 10 300 python -u tools/exp_spmm_k.py powerlaw,uniform > $out/spmm_k_tail.jsonl 2>&1 || { tail -20 $out/spmm_k_tail.jsonl; exit 1; }
grep '^{' $out/spmm_k_notail.jsonl; grep '^{' $out/spmm_k_tail.jsonl
timeout -k 10 500 python -u tools/exp_partition.py > $out/partition.jsonl 2>&1 || { tail -20 $out/partition.jsonl; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r04/partition.jsonl"):
    if l.startswith("{"):
        r = json.loads(l)
        print(r["P"], r["hub_weight"], r["slowest_ms"], r["mean_ms"], r["slowest_over_mean"], [(b["ms"], b["hub_rows"]) for b in r["blocks"]])
PY
