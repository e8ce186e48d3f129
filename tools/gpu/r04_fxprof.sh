#!/bin/bash
# Late round 4: PMC of the dense kernels with the pre-split fused layer (the default), then the
# training-step profiles (tools/gpu/train_prof.sh) at the same head.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r04/pmc_dense_fx bash tools/gpu/pmc_nt.sh > /dev/null && \
python3 tools/pmc_dense_summary.py gpurun_out/r04/pmc_dense_fx --out gpurun_out/r04/pmc_dense_fx/pmc_dense_kernels.json > gpurun_out/r04/pmc_dense_fx/summary.txt 2>&1; \
cat gpurun_out/r04/pmc_dense_fx/summary.txt | cut -c1-250 && \
bash tools/gpu/train_prof.sh
