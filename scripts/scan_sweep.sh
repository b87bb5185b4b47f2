#!/bin/bash
# Scan-kernel sweep on the GPU box: token-major (cost-model segments and forced segment
# counts) vs the channel-major v5 kernel.  Output: gpurun_out/sweep/*.jsonl
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sweep
O=gpurun_out/sweep
T="timeout -k 10 300"
$T python scripts/bench_scan.py --layout tm --batches 1 2 4 8 16 32 64 128 > $O/tm_auto.jsonl
for S in 1 4 16 64; do
  VM_SCAN_SEGMENTS=$S $T python scripts/bench_scan.py --layout tm --batches 1 8 32 > $O/tm_s$S.jsonl
done
$T python scripts/bench_scan.py --layout cm --batches 1 8 32 > $O/cm_v5.jsonl
echo sweep done
