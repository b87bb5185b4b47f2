#!/bin/bash
# Time every scan variant (separate processes: the variant is latched on first use).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in ${VARIANTS:-0 1 3 4}; do
  VM_SCAN_VARIANT=$v timeout -k 10 120 python scripts/bench_scan.py --batches ${BATCHES:-1 4 8} || exit $?
done
