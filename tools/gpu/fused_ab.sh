#!/bin/bash
# A/B of the fused output layer: the committed library (tools/abtest/lib_before.so, loaded via
# GCG_LIB) against the working tree's, alternating, twice each.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for i in 1 2; do
  echo "== before"; GCG_LIB=tools/abtest/lib_before.so timeout -k 10 200 python -u tools/exp_fused_one.py || exit 1
  echo "== after"; timeout -k 10 200 python -u tools/exp_fused_one.py || exit 1
done
