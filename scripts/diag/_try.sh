set -o pipefail
for v in product lin32 product lin32; do
  timeout -k 10 120 python -u scripts/diag/variant_linear.py $v 2>&1 | grep '{' || exit 1
done
