#!/bin/bash
# GPU test suite + smoke on the in-tree build, logs under gpurun_out/$TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r5t}; mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > "$OUT/gpu_tests.log" 2>&1
rc=$?; tail -15 "$OUT/gpu_tests.log"; echo "tests rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; tail -3 "$OUT/smoke.log"; echo "smoke rc=$rc"
exit $rc
