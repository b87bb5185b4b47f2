#!/bin/bash
# Round 6: kernel traces of the 1344-clip step (step_ab.py, 2 reps) with the product
# library and with the dtp_dyn5 variant (bench scan at 96 VGPRs): does add + RMSNorm
# run faster beside the scan once it has registers there?
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp VARIANT_DIR=ab
O=gpurun_out/${TAG:-r06x}
mkdir -p $O
for v in product dtp_dyn5; do
  a=""; [ "$v" != product ] && a="--lib=$v"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o step -- python scripts/diag/step_ab.py --batch=1344 --reps=2 $a > $O/$v.log 2>&1 || { tail $O/$v.log; exit 1; }
  grep ms_per_step $O/$v.log
done
