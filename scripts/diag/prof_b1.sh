#!/bin/bash
# rocprofv3 kernel stats of 10 eager B=1 chunks, channel-major vs token-major mixer.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
for lay in ${LAYS:-cm tm}; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_b1_$lay -o run -- python -u scripts/diag/b1_chunk_eager.py $lay > gpurun_out/prof_b1_$lay.log 2>&1 || { echo "prof $lay failed"; tail -5 gpurun_out/prof_b1_$lay.log; exit 1; }
done
echo ok
