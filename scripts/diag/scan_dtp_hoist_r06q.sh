#!/bin/bash
# Round 6: the chunked scan's dt-block x_dbl loads issued with the start-up loads (one
# round trip fewer per 16 steps) against the committed HEAD build (tools/probes/ab/base_head,
# VARIANT_DIR=ab build_variant.py --rev HEAD base_head): scan parity tests, then the B = 1
# chunk graph alternating ("^ " = this build, "^ lib=..." = HEAD).  Ran against the working
# tree before commit fe2d7dc (the hoist was reverted there, never committed: DESIGN §7).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06q}
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_model.py -k "scan or dtproj or graph_replay or c5_ or chunk" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do for v in "" lib=tools/probes/ab/base_head/libvideomamba_hip.so; do
  timeout -k 10 200 python -u scripts/diag/b1_chunk_graph.py 100 $v >> $O/graph.txt 2>&1 || { tail $O/graph.txt; exit 1; }
  echo "^ $v" >> $O/graph.txt
done; done
grep -A1 "graph replays" $O/graph.txt
