#!/bin/bash
# Small-batch scan: channel-major time-parallel vs token-major segmented (cost-model
# segments), B = 1..64 at D=1152, L=3137.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/b1scan
O=gpurun_out/b1scan/small_batch.txt
: > $O
for lay in cm tm; do
  timeout -k 10 200 python scripts/bench_scan.py --layout $lay --batches 1 2 4 8 16 32 64 --reps 20 | python -c "
import json,sys
for l in sys.stdin: r=json.loads(l); print('$lay', r['shape'].split()[0], r['avg_us'], r['us_per_clip_layer'])" >> $O || exit 1
done
cat $O
