#!/bin/bash
# Round 6: options.stream_post_add (the residual add issued after out_proj, in the scan's
# phase; the next pre phase only normalises): tests, then the 1344-clip step with it on and
# off, alternating in separate processes, then a kernel trace of each.  Ran at commit
# 6ca05ae (the option and its kernels were reverted after it: DESIGN §7).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06y}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_model.py -k "residual_add or post_add or batch_streams or bench_batch or add_norm or world2" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do for v in true false; do
  timeout -k 10 300 python scripts/diag/step_ab.py --batch=1344 --reps=3 --opt=stream_post_add=$v >> $O/step.jsonl 2> $O/step.err || { tail $O/step.err; exit 1; }
done; done
cat $O/step.jsonl
for v in true false; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o step -- python scripts/diag/step_ab.py --batch=1344 --reps=2 --opt=stream_post_add=$v > $O/prof_$v.log 2>&1 || { tail $O/prof_$v.log; exit 1; }
done
echo done
