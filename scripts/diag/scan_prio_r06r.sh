#!/bin/bash
# Round 6: the chunked scan with the two waves of each SIMD swapping the raised issue
# priority every kPF (ch_prio_toggle) or 2 kPF (ch_prio_toggle2) steps, against the product
# build: the B = 1 chunk graph, alternating (VARIANT_DIR=ab build_variant.py NAME).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06r}
mkdir -p $O
for i in 1 2 3; do for v in product ${VARIANTS:-ch_prio_toggle ch_prio_toggle2}; do for bb in ${BATCHES:-1}; do
  a=""; [ "$v" != product ] && a="lib=tools/probes/ab/$v/libvideomamba_hip.so"
  timeout -k 10 200 python -u scripts/diag/b1_chunk_graph.py 100 $a batch=$bb > $O/g.txt 2>&1 || { tail $O/g.txt; exit 1; }
  echo "$v B=$bb $(grep 'graph replays' $O/g.txt)" >> $O/graph.txt
done; done; done
cat $O/graph.txt
