set -o pipefail
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "one_launch or mixer_layout or token_major" > gpurun_out/t5.log 2>&1; rc=$?; tail -3 gpurun_out/t5.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -u scripts/diag/scan_one_launch.py 2>&1 | grep '{' || exit 1
timeout -k 10 180 python -u scripts/diag/b1_chunk_graph.py 50 2>&1 | grep "graph replays" || exit 1
