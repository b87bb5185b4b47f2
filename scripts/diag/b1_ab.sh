#!/bin/bash
# B = 1 chunk graph A/B of probe builds under tools/probes/ab/<name> (VARIANT_DIR=ab
# build_variant.py): chunk graph replay alternating, three rounds.  VARS="a b ..." TAG=...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-b1ab}
mkdir -p $O
for i in 1 2 3; do for v in $VARS; do
  timeout -k 10 200 python -u scripts/diag/b1_chunk_graph.py 100 lib=tools/probes/ab/$v/libvideomamba_hip.so >> $O/graph.txt 2>&1 || { tail $O/graph.txt; exit 1; }
  echo "^ $v" >> $O/graph.txt
done; done
grep -A1 "graph replays" $O/graph.txt
