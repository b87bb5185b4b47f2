#!/bin/bash
# Round evidence: default bench (with cpu baseline), rocprofv3 kernel stats of the same
# command, and FETCH_SIZE / WRITE_SIZE passes on the scan microbench at the bench shape.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=${ROUND:-r01}
mkdir -p gpurun_out/$R
timeout -k 10 900 python bench.py > gpurun_out/$R/bench.json 2> gpurun_out/$R/bench.err || { echo bench failed; tail gpurun_out/$R/bench.err; exit 1; }
cat gpurun_out/$R/bench.json
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$R/prof -o bench -- python bench.py --no-cpu-baseline > gpurun_out/$R/prof_bench.log 2>&1 || { echo prof failed; tail gpurun_out/$R/prof_bench.log; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d gpurun_out/$R/pmc_$c -o scan -- python scripts/bench_scan.py --batches ${BATCH:-32} --reps 3 > gpurun_out/$R/pmc_$c.log 2>&1 || { echo pmc $c failed; tail gpurun_out/$R/pmc_$c.log; exit 1; }
done
echo evidence done
