#!/bin/bash
# Concurrent batch-slice streams A/B on the headline bench (VM_BATCH_STREAMS=1/2/3).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/streams
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_model.py -k "multistream or graph" > gpurun_out/streams/tests.log 2>&1
tail -3 gpurun_out/streams/tests.log
for n in ${NS:-1 2 3}; do
  VM_BATCH_STREAMS=$n timeout -k 10 400 python bench.py --steps ${STEPS:-6} --warmup 2 --no-cpu-baseline --scan-reps 3 --p50-chunks 5 > gpurun_out/streams/bench_$n.json || exit 1
  python -c "
import json; r=json.load(open('gpurun_out/streams/bench_$n.json')); print('streams=$n', r['value'], r['ms_per_step'])"
done
