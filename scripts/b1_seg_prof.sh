#!/bin/bash
# Per-kernel times of the segmented token-major scan at B=1 for several segment counts.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/b1seg
for s in 32 64 128 256; do
  VM_SCAN_SEGMENTS=$s timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/b1seg/s$s -o run -- python scripts/bench_scan.py --layout tm --batches 1 --reps 20 > gpurun_out/b1seg/s$s.log 2>&1 || exit 1
  f=$(find gpurun_out/b1seg/s$s -name "*kernel_stats.csv" | head -1)
  echo "== S=$s"; grep -v "^\"Name" $f | awk -F, '{print $1, $2, $4}' | grep scan
done
