#!/bin/bash
# PMC passes over tools/exp_dense_one.py (one counter set per run, MI355X_MICROARCH.md slots).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=${OUT:-gpurun_out/pmc_nt}
DRIVER=${DRIVER:-tools/exp_dense_one.py}
mkdir -p $out
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt -o kt -- python3 $DRIVER > $out/kt.log 2>&1 || { tail -5 $out/kt.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA GRBM_GUI_ACTIVE --output-format csv -d $out/p1 -o p1 -- python3 $DRIVER > $out/p1.log 2>&1 || { tail -5 $out/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $out/p2 -o p2 -- python3 $DRIVER > $out/p2.log 2>&1 || { tail -5 $out/p2.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/p3 -o p3 -- python3 $DRIVER > $out/p3.log 2>&1 || { tail -5 $out/p3.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/p4 -o p4 -- python3 $DRIVER > $out/p4.log 2>&1 || { tail -5 $out/p4.log; exit 1; }
find $out -name "*.csv" | head -20
