#!/bin/bash
# PMC passes (one group per pass) for scan variants: occupancy, VALU busy, instruction mix.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc2
mkdir -p $OUT
for v in ${VARIANTS:-6 29}; do
  i=0
  for grp in "MeanOccupancyPerActiveCU" "VALUBusy" \
             "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY" \
             "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    VM_SCAN_VARIANT=$v timeout -k 10 180 rocprofv3 --pmc $grp --output-format csv -d $OUT/v${v}_p$i -o run -- python scripts/bench_scan.py --batches ${BATCH:-8} --reps 3 > $OUT/v${v}_p$i.log 2>&1 || { echo "pass $v/$i failed"; tail -20 $OUT/v${v}_p$i.log; exit 1; }
  done
done
echo done
