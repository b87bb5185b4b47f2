#!/bin/bash
# PMC passes over conv_proj / dt_proj at the bench shape (tools/probes/cp_lab, library kernels only)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_cp
mkdir -p $OUT
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SMEM GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- ./tools/probes/cp_lab 336 only > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -20 $OUT/p$i.log; exit 1; }
done
python - <<'PY'
import csv, glob, collections
for kern in ("conv_proj_kernel", "dt_proj_kernel"):
    vals = collections.defaultdict(list)
    for f in glob.glob("gpurun_out/pmc_cp/p*/**/*counter_collection.csv", recursive=True):
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in csv.DictReader(open(f)):
            if kern in r["Kernel_Name"]:
                per[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
        for c, d in per.items():
            vals[c].append(sum(d.values()) / len(d))
    print(kern)
    for c in sorted(vals):
        print(f"  {c:28s} {sum(vals[c]) / len(vals[c]):.4g}")
PY
