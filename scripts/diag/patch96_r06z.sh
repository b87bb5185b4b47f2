#!/bin/bash
# Round 6: the B = 1 patch embed on 64 x 96 tiles (294 workgroups) against HEAD's 64 x 192
# (147): patch parity tests, the B = 1 chunk graph alternating, and a kernel trace of each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06z}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_model.py -k "patch or graph_replay or model_cases or embed" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do for v in product base_head; do
  a=""; [ "$v" != product ] && a="lib=tools/probes/ab/$v/libvideomamba_hip.so"
  timeout -k 10 200 python -u scripts/diag/b1_chunk_graph.py 100 $a > $O/g.txt 2>&1 || { tail $O/g.txt; exit 1; }
  echo "$v $(grep 'graph replays' $O/g.txt)" >> $O/graph.txt
done; done
cat $O/graph.txt
for v in product base_head; do
  a=""; [ "$v" != product ] && a="lib=tools/probes/ab/$v/libvideomamba_hip.so"
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$v -o run -- python -u scripts/diag/b1_chunk_graph.py 50 $a > $O/prof_$v.log 2>&1 || { tail $O/prof_$v.log; exit 1; }
done
grep -h patch_mfma16 $O/prof_*/run_kernel_stats.csv | cut -d, -f1-4
