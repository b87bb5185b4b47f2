#!/bin/bash
# A/B of token-major scan variants: SGPR B/C (default) vs LDS-staged B/C.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sweep
T="timeout -k 10 300"
$T python scripts/bench_scan.py --layout tm --batches ${BATCHES:-1 32 112 224} > gpurun_out/sweep/tm_sgpr.jsonl
VM_SCAN_SGPR=0 $T python scripts/bench_scan.py --layout tm --batches ${BATCHES:-1 32 112 224} > gpurun_out/sweep/tm_lds.jsonl
for f in tm_sgpr tm_lds; do python - "$f" <<'PY'
import json, sys
f = sys.argv[1]
for l in open(f"gpurun_out/sweep/{f}.jsonl"):
    r = json.loads(l)
    print(f, r["shape"].split()[0], r["avg_us"], r["us_per_clip_layer"], r["frac"])
PY
done
