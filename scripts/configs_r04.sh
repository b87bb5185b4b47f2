#!/bin/bash
# The other BASELINE configs on one GPU (C2 Ti-8f full sequence, M-32f clip shape, C5 long video);
# results under gpurun_out/$R (default r04z).
set -e
export TMPDIR=/tmp
O=gpurun_out/${R:-r04z}; mkdir -p $O
timeout -k 10 300 python bench.py --config ti8 --full-sequence --batch 512 --no-b1 --no-cpu-baseline > $O/c2_ti8.json 2> $O/c2.err || { echo c2 failed; tail $O/c2.err; exit 1; }
cat $O/c2_ti8.json | python -c "import json,sys; d=json.load(sys.stdin); print('C2', d['value'], d['ms_per_step'])"
timeout -k 10 300 python bench.py --config m32 --no-b1 --no-cpu-baseline > $O/m32.json 2> $O/m32.err || { echo m32 failed; tail $O/m32.err; exit 1; }
cat $O/m32.json | python -c "import json,sys; d=json.load(sys.stdin); print('M32', d['value'], d['ms_per_step'])"
timeout -k 10 600 python scripts/bench_long_video.py > $O/long_video.json 2> $O/long_video.err || { echo long video failed; tail $O/long_video.err; exit 1; }
cat $O/long_video.json
