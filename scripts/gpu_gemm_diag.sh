#!/bin/bash
# gemm_big structure diagnostics: 256x256 glds GEMM as is / without the DMA
# wait / without wait and barrier, on the large-v3 encoder shapes; PMC passes.
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT/scripts/probe" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
timeout -k 10 120 ./gemm_diag > $O/gemm_diag.txt 2>&1 || exit 4
cat $O/gemm_diag.txt
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $O/pmc_gdiag1 -o pmc -- $GRAFT_REPO_ROOT/scripts/probe/gemm_diag > $O/pmc_gdiag1.log 2>&1 || exit 5
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA --output-format csv -d $O/pmc_gdiag2 -o pmc -- $GRAFT_REPO_ROOT/scripts/probe/gemm_diag > $O/pmc_gdiag2.log 2>&1 || exit 5
echo pmc done
