#!/bin/bash
# Per-kernel times (rocprofv3 kernel stats) of the split-K conv_proj at B=1 for each variant.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
for v in ${VARS:-product}; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pcv_$v -o run -- python -u scripts/diag/variant_conv.py $v 1 > gpurun_out/pcv_$v.log 2>&1 || { echo "$v failed"; tail -3 gpurun_out/pcv_$v.log; exit 1; }
  grep '{' gpurun_out/pcv_$v.log
  grep -E "conv_xproj_tm|xdbl_dt_tm" gpurun_out/pcv_$v/run_kernel_stats.csv | cut -d, -f1-4
done
