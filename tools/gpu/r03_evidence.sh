#!/bin/bash
# Round-3 evidence: the bench command under rocprofv3 (kernel trace + stats), the SpMM's
# L2->fabric bytes in the mode auto resolves to, and the training-step traces.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
bash tools/gpu/bench_prof.sh || exit 1
bash tools/gpu/pmc_spmm_auto.sh || exit 1
bash tools/gpu/train_prof.sh || exit 1
echo evidence done
