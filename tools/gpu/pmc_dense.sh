#!/bin/bash
# PMC passes (one counter set per run) over tools/exp_dense_one.py: MFMA busy cycles, wave
# cycles, waits and instruction mix of the fused output kernel and the plain MFMA GEMM.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/pmc_dense
mkdir -p $out
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $out/p1 -o p1 -- python3 tools/exp_dense_one.py > $out/p1.log 2>&1 || { tail -5 $out/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $out/p2 -o p2 -- python3 tools/exp_dense_one.py > $out/p2.log 2>&1 || { tail -5 $out/p2.log; exit 1; }
ls -R $out | head -20
