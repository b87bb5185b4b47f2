set -o pipefail
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t7.log 2>&1; rc=$?; tail -2 gpurun_out/t7.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -u scripts/diag/scan_one_launch.py 2>&1 | grep '{' || exit 1
for v in product sc_noahead; do timeout -k 10 120 python -u scripts/diag/variant_scan.py $v 336 2>&1 | grep '{' || exit 1; done
timeout -k 10 180 python -u scripts/diag/b1_chunk_graph.py 50 2>&1 | grep "graph replays" || exit 1
