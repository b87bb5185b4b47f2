cd /root/repo
export TMPDIR=/tmp
for M in 1 0; do
  mkdir -p gpurun_out/prof_pre$M
  VM_DELTA_IN_CONV_PROJ=$M timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_pre$M -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --p50-chunks 3 --scan-reps 5 > gpurun_out/prof_pre$M/bench.log 2>&1 || exit $?
done
