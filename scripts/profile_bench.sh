#!/bin/bash
# rocprofv3 kernel-trace + stats of a short bench run (no PMC, no trace domains).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_${TAG:-bench}
mkdir -p $OUT
timeout -k 10 ${TMO:-600} rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python bench.py ${BENCH_ARGS:---steps 5 --warmup 2 --no-cpu-baseline --p50-chunks 3 --scan-reps 5} > $OUT/bench.log 2>&1
rc=$?; tail -3 $OUT/bench.log; exit $rc
