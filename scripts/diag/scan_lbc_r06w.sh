#!/bin/bash
# Round 6: the one-launch chunked scan with the block's B|C rows staged in LDS as fp32 (LBC)
# against the committed HEAD build (tools/probes/ab/base_head): scan / mixer / model parity
# tests, then the B = 1 and B = 2 chunk graphs alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06w}
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_model.py -k "scan or dtproj or graph_replay or c5_ or chunk or stream" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do for v in product base_head; do for bb in 1 2; do
  a=""; [ "$v" != product ] && a="lib=tools/probes/ab/$v/libvideomamba_hip.so"
  timeout -k 10 200 python -u scripts/diag/b1_chunk_graph.py 100 $a batch=$bb > $O/g.txt 2>&1 || { tail $O/g.txt; exit 1; }
  echo "$v B=$bb $(grep 'graph replays' $O/g.txt)" >> $O/graph.txt
done; done; done
cat $O/graph.txt
