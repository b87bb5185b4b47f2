#!/bin/bash
# Round evidence: the default bench (with CPU baseline), rocprofv3 kernel stats of the same
# command, kernel stats of the scan microbench alone at the bench shape (the roofline
# kernel), FETCH_SIZE / WRITE_SIZE / SQ counter passes on that microbench, the same
# FETCH/WRITE passes on a calibration kernel with the scan's access pattern and a known byte
# count (tools/probes/scan_lab calib), the C5 long-video run, the C2 (Ti-8f full sequence)
# and M-32f bench lines and the B=1 graph-replay chunk profile.  PART=1: bench + its profile; PART=2: the rest (one gpurun call each).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=${ROUND:-r03}
B=${BATCH:-448}
DTP=${DTP:---dtp}
O=gpurun_out/$R
mkdir -p $O
if [ "${PART:-1}" = 1 ]; then
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python bench.py --no-cpu-baseline > $O/prof_bench.log 2>&1 || { echo prof failed; tail $O/prof_bench.log; exit 1; }
echo part 1 done
exit 0
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_scan -o scan -- python scripts/bench_scan.py --batches $B --reps 20 $DTP > $O/prof_scan.log 2>&1 || { echo scan prof failed; tail $O/prof_scan.log; exit 1; }
for c in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VALU_TRANS_F32 SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"; do
  tag=$(echo $c | cut -d' ' -f1)
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $O/pmc_$tag -o scan -- python scripts/bench_scan.py --batches $B --reps 3 $DTP > $O/pmc_$tag.log 2>&1 || { echo pmc $c failed; tail $O/pmc_$tag.log; exit 1; }
done
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $O/calib_$c -o calib -- ./tools/probes/scan_lab $B 2 3137 calib > $O/calib_$c.log 2>&1 || { echo calib $c failed; tail $O/calib_$c.log; exit 1; }
done
timeout -k 10 600 python scripts/bench_long_video.py > $O/long_video.json 2> $O/long_video.err || { echo long video failed; tail $O/long_video.err; exit 1; }
cat $O/long_video.json
timeout -k 10 300 python bench.py --config ti8 --full-sequence --batch 512 --no-b1 --no-cpu-baseline > $O/c2_ti8.json 2> $O/c2.err || { echo c2 failed; tail $O/c2.err; exit 1; }
timeout -k 10 300 python bench.py --config m32 --no-b1 --no-cpu-baseline > $O/m32.json 2> $O/m32.err || { echo m32 failed; tail $O/m32.err; exit 1; }
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_b1_graph -o run -- python -u scripts/diag/b1_chunk_graph.py 20 > $O/prof_b1_graph.log 2>&1 || { echo b1 prof failed; tail $O/prof_b1_graph.log; exit 1; }
grep "graph replays" $O/prof_b1_graph.log
echo evidence done
