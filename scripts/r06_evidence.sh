#!/bin/bash
# Round-6 evidence in one call: the default bench line, the rocprofv3 kernel summary of the
# same command (the in-step scan trace bench.py reads), the B = 1 graph-replay kernel trace,
# and the C2 / C4-shape / C5 lines.  Every GPU step has its own time limit; the first
# failure ends the call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06j}
mkdir -p $O
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail $O/bench.err; exit 1; }
tail -c 600 $O/bench.json; echo
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python bench.py --no-cpu-baseline > $O/prof_bench.log 2>&1 || { echo prof failed; tail $O/prof_bench.log; exit 1; }
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_b1 -o run -- python -u scripts/diag/b1_chunk_graph.py 50 > $O/prof_b1.log 2>&1 || { echo b1 prof failed; tail $O/prof_b1.log; exit 1; }
grep "graph replays" $O/prof_b1.log
[ "${PART2:-1}" = 1 ] || exit 0
timeout -k 10 600 python scripts/bench_long_video.py > $O/long_video.json 2> $O/long_video.err || { echo long video failed; tail $O/long_video.err; exit 1; }
tail -c 300 $O/long_video.json; echo
timeout -k 10 300 python bench.py --config ti8 --full-sequence --batch 512 --no-b1 --no-cpu-baseline > $O/c2_ti8.json 2> $O/c2.err || { echo c2 failed; tail $O/c2.err; exit 1; }
timeout -k 10 400 python bench.py --config m32 --no-b1 --no-cpu-baseline > $O/m32.json 2> $O/m32.err || { echo m32 failed; tail $O/m32.err; exit 1; }
python -c "
import json
for f in ['c2_ti8', 'm32']:
    d = json.load(open('$O/' + f + '.json'))
    print(f, d['value'], d['ms_per_step'])
"
echo evidence done
