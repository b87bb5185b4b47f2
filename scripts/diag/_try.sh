set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t2.log 2>&1; rc=$?; tail -4 gpurun_out/t2.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 120 python -u scripts/diag/variant_conv.py product 1 2 4 8 2>&1 | grep '{' || exit 1
timeout -k 10 120 python -u scripts/diag/variant_conv.py cp_splitk 1 2 4 8 2>&1 | grep '{' || exit 1
timeout -k 10 180 python -u scripts/diag/b1_chunk_graph.py 50 2>&1 | grep "graph replays" || exit 1
