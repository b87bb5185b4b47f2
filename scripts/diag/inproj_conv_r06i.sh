#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${TAG:-r06i}
mkdir -p $O
timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_parity.py -k in_proj_conv_proj > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do for v in product ${VARIANTS:-ic_prev ic_prio ic_norenum}; do
  timeout -k 10 120 python scripts/diag/inproj_conv_bench.py $v 1 >> $O/ab.jsonl 2>/dev/null || exit 1
done; done
cat $O/ab.jsonl
