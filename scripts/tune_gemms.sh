#!/bin/bash
# Record TunableOp results for the projection GEMM shapes the bench / tests use (run on the
# GPU box; copies the results file to gpurun_out/ so it can be committed).
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for B in ${BATCHES:-1 32 224}; do
  VM_GEMM_TUNING=tune timeout -k 10 900 python bench.py --batch $B --steps 1 --warmup 1 \
    --p50-chunks 1 --scan-reps 1 --no-cpu-baseline > gpurun_out/tune_b$B.json
  echo "tuned B=$B"
done
cp videomamba_amd/tuning/tunableop_gfx950.csv gpurun_out/tunableop_gfx950.csv
wc -l gpurun_out/tunableop_gfx950.csv
