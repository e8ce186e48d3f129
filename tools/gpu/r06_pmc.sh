#!/bin/bash
# round 6: the compile tests (incl. the non-symmetric operator), then PMC passes over the output
# layer's kernels at the head (tools/gpu/pmc_nt.sh) and their summary.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r06p
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_ops_gpu.py > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
OUT=$out/pmc timeout -k 10 700 bash tools/gpu/pmc_nt.sh > $out/pmc.log 2>&1 || { tail -20 $out/pmc.log; exit 1; }
python tools/pmc_dense_summary.py $out/pmc --out $out/pmc_dense_kernels.json > /dev/null
