#!/bin/bash
# Round 6: the in_proj + conv kernel's x_dbl partials summed by the row tile's last
# arriving split (one launch, ABI v15) against the second reduce launch: parity tests,
# then the B = 1 chunk graph alternating, then a kernel trace of the product form.
# Ran against commit 90c4891 (the in-kernel sum and b1_chunk_graph.py's ic_sum= hook; reverted).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06n}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_model.py -k "in_proj_conv or graph_replay or c5_" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do for v in ic_sum=kernel ic_sum=launch; do
  timeout -k 10 200 python -u scripts/diag/b1_chunk_graph.py 100 $v >> $O/graph.txt 2>&1 || { tail $O/graph.txt; exit 1; }
done; done
grep "graph replays" $O/graph.txt
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o b1 -- python3 $GRAFT_REPO_ROOT/scripts/diag/b1_chunk_graph.py 100 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
find $GRAFT_REPO_ROOT/$O/prof -name "*kernel_stats.csv" | head -3
