#!/bin/bash
# add + RMSNorm rows per wave: bitwise tests, then the 1344-clip step per variant, alternating
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${TAG:-r06k}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py::test_add_rms_rows_per_wave_is_bitwise_one_row_per_wave "tests/test_gpu_model.py::test_c3_bench_batch_clips_bitwise_equal_small_batch_and_oracle[1344]" > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do for v in product ${VARIANTS:-an_rpw1 an_rpw4 an_rpw16}; do
  if [ $v = product ]; then a=""; else a="--lib=$v"; fi
  VARIANT_DIR=ab timeout -k 10 200 python scripts/diag/step_ab.py $a --batch=1344 --reps=3 >> $O/step.jsonl 2>/dev/null || exit 1
  tail -1 $O/step.jsonl
done; done
