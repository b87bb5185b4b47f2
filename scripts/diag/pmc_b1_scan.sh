#!/bin/bash
# Kernel stats + SQ counters of the token-major scan micro-benchmark at B=1 (M-16f shape).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/pmc_b1
mkdir -p $O
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python -u scripts/bench_scan.py --batches 1 --layout tm --reps 20 > $O/stats.log 2>&1 || { echo stats failed; tail $O/stats.log; exit 1; }
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d $O/sq -o run -- python -u scripts/bench_scan.py --batches 1 --layout tm --reps 3 > $O/sq.log 2>&1 || { echo sq failed; tail $O/sq.log; exit 1; }
timeout -k 10 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD --output-format csv -d $O/grbm -o run -- python -u scripts/bench_scan.py --batches 1 --layout tm --reps 3 > $O/grbm.log 2>&1 || { echo grbm failed; tail $O/grbm.log; exit 1; }
cat $O/stats.log | tail -2
echo ok
