#!/bin/bash
# B=1 latency probes: scan variants at B=1 (channel-major) and the chunk p50 with and
# without the tuned GEMM table.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/p50
for v in 0 3 4 5 14 15 16 17; do
  VM_SCAN_VARIANT=$v timeout -k 10 120 python scripts/bench_scan.py --layout cm --batches 1 2 --reps 30 > gpurun_out/p50/v$v.jsonl || exit 1
  python -c "
import json
for l in open('gpurun_out/p50/v$v.jsonl'):
    r = json.loads(l); print('variant $v', r['shape'].split()[0], r['avg_us'])"
done
for g in 1 0; do
  VM_GEMM_TUNING=$g timeout -k 10 300 python bench.py --batch 1 --steps 3 --warmup 2 --p50-chunks 40 --scan-reps 3 --no-cpu-baseline > gpurun_out/p50/bench_g$g.json || exit 1
  python -c "
import json; r = json.load(open('gpurun_out/p50/bench_g$g.json')); print('gemm_tuning=$g p50', r['chunk_p50_ms'], 'ms/step', r['ms_per_step'])"
done
