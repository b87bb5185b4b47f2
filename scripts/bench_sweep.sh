#!/bin/bash
# Whole-model bench at several per-GPU batches (no CPU baseline): gpurun_out/bsweep/*.json
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/bsweep
for B in ${BATCHES:-32 112 224}; do
  timeout -k 10 600 python bench.py --batch $B --steps ${STEPS:-5} --warmup 2 --p50-chunks 5 \
    --scan-reps 10 --no-cpu-baseline > gpurun_out/bsweep/b$B.json
  echo "B=$B $(python -c "import json;r=json.load(open('gpurun_out/bsweep/b$B.json'));print(r['value'], r['ms_per_step'], r['roofline']['avg_us'], r['roofline']['layout'])")"
done
