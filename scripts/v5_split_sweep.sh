#!/bin/bash
# Channel-major scan at small batches (the B = 1 latency path), v5 against its state-split
# forms (VM_SCAN_VARIANT 30-35: 16 states over 2 or 4 waves per channel).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for V in ${VARIANTS:-0 30 31 32 33 34 35 36 37 0}; do
  VM_SCAN_VARIANT=$V timeout -k 10 120 python scripts/bench_scan.py --batches 1 2 4 8 --layout cm --reps 50 || exit $?
done
