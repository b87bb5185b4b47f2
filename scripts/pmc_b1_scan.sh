#!/bin/bash
# PMC passes over the channel-major (small-batch) scan at B=1, D=1152, L=3137: where the
# B=1 streaming chunk's scan time goes (issue vs waiting).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_b1
mkdir -p $OUT
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/p$i -o run -- python scripts/bench_scan.py --layout cm --batches 1 --reps 5 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -20 $OUT/p$i.log; exit 1; }
done
python - <<'PY'
import csv, glob, collections
vals = collections.defaultdict(list)
for f in glob.glob("gpurun_out/pmc_b1/p*/**/*counter_collection.csv", recursive=True):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        if "scan_v5" in r["Kernel_Name"]:
            per[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    for c, d in per.items():
        vals[c].append(sum(d.values()) / len(d))
for c in sorted(vals):
    print(f"{c:28s} {sum(vals[c]) / len(vals[c]):.4g}")
PY
