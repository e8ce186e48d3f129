#!/bin/bash
# Round 4: PMC passes over the bf16x6 pre-split NT GEMM, two tiles.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for cfg in ${NT3_CFGS:-"2,1,4,1,2" "2,2,4,1,2"}; do
  tag=$(echo $cfg | tr ',' '_')
  GCG_NT3_CFG=$cfg OUT=gpurun_out/r04/nt3pmc/$tag DRIVER=tools/exp_nt3_one.py bash tools/gpu/pmc_nt.sh > /dev/null || exit 1
  python3 tools/pmc_dense_summary.py gpurun_out/r04/nt3pmc/$tag --out gpurun_out/r04/nt3pmc/$tag.json > /dev/null || exit 1
  python3 -c "
import json; r=json.load(open('gpurun_out/r04/nt3pmc/$tag.json'))
for k,v in r.items(): print('$cfg', k[:60], {x: y for x, y in v.items() if x != 'counters_per_dispatch'}, {c: v['counters_per_dispatch'].get(c) for c in ('SQ_WAVE_CYCLES','SQ_BUSY_CYCLES','SQ_INSTS_MFMA','SQ_INSTS_VALU','SQ_INSTS_LDS','SQ_LDS_IDX_ACTIVE','SQ_LDS_BANK_CONFLICT','SQ_WAVES')})
"
done
