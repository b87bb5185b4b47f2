#!/bin/bash
# Round 6: the in_proj + conv epilogue path (vm_in_proj_conv_proj_fwd) — its bitwise tests,
# then the B = 1 graph chunk with it off / on, alternating, then a kernel trace with it on.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06b}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_gpu_parity.py -k "in_proj_conv_proj" > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for i in 1 2; do
  for c in 0 2; do
    timeout -k 10 200 python -u scripts/diag/b1_chunk_graph.py 100 in_proj_conv_clips=$c >> $O/ab.txt 2>&1 || { echo ab failed; tail $O/ab.txt; exit 1; }
  done
done
cat $O/ab.txt | grep "graph replays"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_b1 -o run -- python -u scripts/diag/b1_chunk_graph.py 20 > $O/prof_b1.log 2>&1 || { echo prof failed; tail $O/prof_b1.log; exit 1; }
echo done
