#!/bin/bash
# Token-major (segmented) scan at B=1, D=1152, L=3137: SGPR vs LDS B/C staging over segment
# counts, HIP-event time per call (three launches: summary, carry, final).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for sg in 1 0; do
  for s in 16 32 64 128 256; do
    VM_SCAN_SGPR=$sg VM_SCAN_SEGMENTS=$s timeout -k 10 100 python scripts/bench_scan.py --layout tm --batches 1 --reps 30 2>/dev/null | python -c "
import json,sys
for l in sys.stdin:
    if l.startswith('{'): r=json.loads(l); print('sgpr=$sg S=$s', r['avg_us'])" || exit 1
  done
done
