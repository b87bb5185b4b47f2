#!/bin/bash
# B=1 scan options at D=1152, L=3137: channel-major time-parallel (default at B=1) vs the
# token-major channel-per-lane kernel at several segment counts, SGPR vs LDS B/C.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/b1scan
O=gpurun_out/b1scan/sweep.txt
: > $O
timeout -k 10 120 python scripts/bench_scan.py --layout cm --batches 1 2 4 --reps 30 | python -c "
import json,sys
for l in sys.stdin: r=json.loads(l); print('cm', r['shape'].split()[0], r['avg_us'])" >> $O || exit 1
for sg in 1 0; do for s in 16 32 64; do
  VM_SCAN_SGPR=$sg VM_SCAN_SEGMENTS=$s timeout -k 10 120 python scripts/bench_scan.py --layout tm --batches 1 2 4 --reps 30 | python -c "
import json,sys
for l in sys.stdin: r=json.loads(l); print('tm sgpr=$sg seg=$s', r['shape'].split()[0], r['avg_us'])" >> $O || exit 1
done; done
cat $O
