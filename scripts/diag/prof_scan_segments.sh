#!/bin/bash
# rocprofv3 kernel stats of the token-major scan at B=1 for several forced segment counts.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
for S in ${SEGS:-32 64 128 228}; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/scanseg/s$S -o run -- python -u scripts/bench_scan.py --batches ${B:-1} --layout tm --reps 20 --segments $S > gpurun_out/scanseg/s$S.log 2>&1 || { echo "S=$S failed"; tail -5 gpurun_out/scanseg/s$S.log; exit 1; }
done
echo ok
