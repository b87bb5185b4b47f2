for v in ${VARIANTS:-0 18 19}; do
  VM_SCAN_VARIANT=$v timeout -k 10 100 python scripts/bench_scan.py --layout cm --batches 1 2 4 --reps 20 2>/dev/null | python -c "
import json,sys
for l in sys.stdin:
    if l.startswith('{'): r=json.loads(l); print('variant $v', r['shape'].split()[0], r['avg_us'])" || exit 1
done
