#!/bin/bash
# PMC passes over the single-pass scan at B = 336: the plain kernel (dt rows) and the
# dt_proj-in-scan kernel.  One counter group per rocprofv3 pass (gfx950 block limits).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_dtp
mkdir -p $OUT
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_MFMA SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  for mode in plain dtp; do
    flag=""; [ $mode = dtp ] && flag="--dtp"
    timeout -k 10 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/${mode}_p$i -o run -- python3 scripts/diag/variant_scan.py product 336 $flag > $OUT/${mode}_p$i.log 2>&1 || { echo "pass $mode $i failed"; tail -20 $OUT/${mode}_p$i.log; exit 1; }
  done
done
python3 scripts/pmc_summary.py $OUT --kernel scan_seq
