#!/bin/bash
# Round-4 GPU session: GPU tests + smoke, then the default bench and its rocprofv3 kernel
# stats (ROUND tag in $R).  Every GPU step under its own timeout; stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=${R:-r04}
O=gpurun_out/$R
mkdir -p $O
if [[ ${STEPS:-tests,bench,prof} == *tests* ]]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo tests failed; tail -30 $O/gpu_tests.log; exit 1; }
  tail -2 $O/gpu_tests.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
fi
if [[ ${STEPS:-tests,bench,prof} == *bench* ]]; then
  timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail $O/bench.err; exit 1; }
  cat $O/bench.json
fi
if [[ ${STEPS:-tests,bench,prof} == *prof* ]]; then
  timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python bench.py --no-cpu-baseline > $O/prof_bench.log 2>&1 || { echo prof failed; tail $O/prof_bench.log; exit 1; }
  echo prof done
fi
echo session done
