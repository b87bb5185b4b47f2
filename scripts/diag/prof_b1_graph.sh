#!/bin/bash
# rocprofv3 kernel stats of 20 hipGraph-replayed B=1 M-16f chunks (the chunk_p50 path).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_b1_graph -o run -- python -u scripts/diag/b1_chunk_graph.py 20 > gpurun_out/prof_b1_graph.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/prof_b1_graph.log; exit 1; }
grep "graph replays" gpurun_out/prof_b1_graph.log
echo ok
