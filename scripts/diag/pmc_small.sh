#!/bin/bash
# SQ counters of the small-batch kernels (scripts/diag/small_batch_kernels.py, B=1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/pmc_small
mkdir -p $O
export BATCHES="${BATCHES:-1}"
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d $O/sq -o run -- python -u scripts/diag/small_batch_kernels.py > $O/sq.log 2>&1 || { echo sq failed; tail $O/sq.log; exit 1; }
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $O/mem -o run -- python -u scripts/diag/small_batch_kernels.py > $O/mem.log 2>&1 || { echo mem failed; tail $O/mem.log; exit 1; }
echo ok
