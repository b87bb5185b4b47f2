#!/bin/bash
# Round 6: the fused in_proj's K loop as 32-wide steps through 4 stage buffers (3 in
# flight) with the epilogue operands issued 3 steps early, against the 2-buffer 64-wide
# form (ic_2buf = the previous revision): parity tests, the front alone alternating, then
# the B = 1 chunk graph.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06l}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "in_proj_conv_proj" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do for v in product ${VARIANTS:-ic_2buf}; do for b in 1 2; do
  timeout -k 10 120 python scripts/diag/inproj_conv_bench.py $v $b >> $O/ab.jsonl 2>/dev/null || exit 1
done; done; done
cat $O/ab.jsonl
for i in 1 2; do
  timeout -k 10 200 python -u scripts/diag/b1_chunk_graph.py 100 >> $O/graph.txt 2>&1 || { tail $O/graph.txt; exit 1; }
done
grep "graph replays" $O/graph.txt
