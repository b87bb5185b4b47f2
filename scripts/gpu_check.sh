#!/bin/bash
# One GPU-box session: smoke, GPU tests, short bench.  Stops at the first fault/abort/
# timeout (exit codes other than 0 = pass, 1 = test failures).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {  # run <name> <timeout-s> <cmd...>
  local name=$1 tmo=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$tmo" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
STEPS=${STEPS:-smoke,tests,bench}
[[ $STEPS == *smoke* ]] && run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
[[ $STEPS == *tests* ]] && run gpu_tests ${TEST_TMO:-900} python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-}
[[ $STEPS == *bench* ]] && run bench 600 python -u bench.py ${BENCH_ARGS:---steps 10 --warmup 3}
exit 0
