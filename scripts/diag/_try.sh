set -o pipefail
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t3.log 2>&1; rc=$?; tail -3 gpurun_out/t3.log; [ $rc -le 1 ] || exit $rc
for v in product ch_xcd product ch_xcd; do
  timeout -k 10 120 python -u scripts/diag/variant_scan.py $v 1 2 2>&1 | grep '{' || exit 1
done
