set -o pipefail
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t8.log 2>&1; rc=$?; tail -2 gpurun_out/t8.log; [ $rc -eq 0 ] || exit $rc
for v in product sc_nogate product sc_nogate product sc_nogate; do timeout -k 10 120 python -u scripts/diag/variant_scan.py $v 336 1 2>&1 | grep '{' || exit 1; done
