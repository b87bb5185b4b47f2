#!/bin/bash
# Kernel trace of the B=1 streaming chunk (VideoMamba-M 16f) — where the p50 latency goes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/b1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/b1/trace -o run -- \
  python bench.py --batch 1 --steps 3 --warmup 2 --p50-chunks 5 --scan-reps 2 --no-cpu-baseline > gpurun_out/b1/bench.json 2> gpurun_out/b1/err.log || exit 1
find gpurun_out/b1/trace -name "*kernel_stats.csv" -exec cp {} gpurun_out/b1/kernel_stats.csv \;
head -25 gpurun_out/b1/kernel_stats.csv
