#!/bin/bash
# Round 6: the 1344-clip step (two locked sub-batch streams) with the bench scan compiled
# for 96 VGPRs (dynamic LDS keeps it at 4 waves per SIMD, leaving registers for the other
# stream's add + RMSNorm waves: variant dtp_dyn5) against the product, alternating; then
# both scans alone at B = 672 (bench.scan_roofline).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp VARIANT_DIR=ab
O=gpurun_out/${TAG:-r06u}
mkdir -p $O
for i in 1 2 3; do for v in product ${VARIANTS:-dtp_dyn5}; do
  a=""; [ "$v" != product ] && a="--lib=$v"
  timeout -k 10 300 python scripts/diag/step_ab.py --batch=${BATCH:-1344} --reps=3 $a >> $O/step.jsonl 2> $O/step.err || { tail $O/step.err; exit 1; }
done; done
cat $O/step.jsonl
