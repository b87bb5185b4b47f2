#!/bin/bash
# Round 6: clips per GPU for the C3 bench step (two sub-batch streams, phase lock): 1344
# (the default) against 2016 and 2688, alternating, --no-b1 --no-cpu-baseline.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06p}
mkdir -p $O
for i in 1 2; do for b in 1344 2016 2688; do
  timeout -k 10 300 python -u bench.py --batch $b --steps 10 --warmup 3 --no-b1 --no-cpu-baseline --scan-reps 5 > $O/b$b.$i.json 2> $O/b$b.$i.err || { tail -20 $O/b$b.$i.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/b$b.$i.json').read().strip().splitlines()[-1]); print($b, d['value'], d['ms_per_step'])"
done; done
