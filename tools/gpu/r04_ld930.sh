#!/bin/bash
# Round 4: row stride of the C = 930 operand (and K = 928 / 300 controls), World uniform +
# power-law, interleaved on one box.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r04/${LD_OUT:-ld930}
mkdir -p $out
LD_CASES="${LD_CASES:-930:932,936,944,960,992;928:928,932;300:304,320}" timeout -k 10 600 python -u tools/exp_ld_k.py uniform,powerlaw > $out/ld.jsonl 2> $out/ld.err || { tail -20 $out/ld.err; exit 1; }
cat $out/ld.jsonl
