#!/bin/bash
# PMC passes over vm_linear_fwd at the B=1 chunk projection shapes (scripts/diag/variant_linear.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_linear
mkdir -p $OUT
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_MFMA" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/lin_p$i -o run -- python3 scripts/diag/variant_linear.py product > $OUT/lin_p$i.log 2>&1 || { echo "pass $i failed"; tail -20 $OUT/lin_p$i.log; exit 1; }
done
python3 scripts/pmc_summary.py $OUT --kernel linear_kernel
