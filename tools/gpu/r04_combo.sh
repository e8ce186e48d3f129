#!/bin/bash
# One box: the column-sum check (r04_colsum.sh), then the final evidence (r04_final2.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu/r04_colsum.sh && bash tools/gpu/r04_final2.sh
