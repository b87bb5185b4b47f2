#!/bin/bash
# PMC passes on the scan microbench (one counter group per pass; no trace domains).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc
mkdir -p $OUT
for v in ${VARIANTS:-1 4}; do
  i=0
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY" \
             "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
             "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    VM_SCAN_VARIANT=$v timeout -k 10 180 rocprofv3 --pmc $grp --output-format csv -d $OUT/v${v}_p$i -o run -- python scripts/bench_scan.py --batches ${BATCH:-8} --reps 3 > $OUT/v${v}_p$i.log 2>&1 || { echo "pass $v/$i failed"; tail -20 $OUT/v${v}_p$i.log; exit 1; }
  done
done
echo done
