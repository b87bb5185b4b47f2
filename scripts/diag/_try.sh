set -o pipefail
for b in 288 336 392 448 504; do
  timeout -k 10 300 python -u bench.py --batch $b --steps 8 --warmup 3 --no-cpu-baseline --p50-chunks 5 --scan-reps 3 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($b, d['value'], d['ms_per_step'])" || exit 1
done
