#!/bin/bash
# Token-major scan: packed state pairs (default) vs scalar form (VM_SCAN_PK=0), after the
# token-major parity tests.  Output under gpurun_out/pk/.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pk
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "token_major or fixture" > gpurun_out/pk/tests.log 2>&1
B="${BATCHES:-1 32 336}"
timeout -k 10 300 python scripts/bench_scan.py --layout tm --batches $B > gpurun_out/pk/pk1.jsonl
VM_SCAN_PK=0 timeout -k 10 300 python scripts/bench_scan.py --layout tm --batches $B > gpurun_out/pk/pk0.jsonl
for f in pk1 pk0; do python - "$f" <<'PY'
import json, sys
f = sys.argv[1]
for l in open(f"gpurun_out/pk/{f}.jsonl"):
    r = json.loads(l)
    print(f, r["shape"].split()[0], r["avg_us"], r["us_per_clip_layer"], r["frac"])
PY
done
