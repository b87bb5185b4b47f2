#!/bin/bash
# Round-6 final evidence in one call: smoke, the full -m gpu suite, then r06_evidence.sh
# (bench line, its rocprofv3 kernel summary, the B = 1 graph trace, C5 / C2 / C4-shape).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06v}
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo tests failed; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
TAG=${TAG:-r06v} bash scripts/r06_evidence.sh
