#!/bin/bash
# Round-4 measurement, part 1: GPU tests + smoke on the in-tree build, then a rocprofv3 kernel
# trace of exactly the driver's bench command and the trace-vs-bench check.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r4g}; mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests > gpurun_out/$TAG/tests.log 2>&1
rc=$?; tail -3 gpurun_out/$TAG/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/$TAG/smoke.log 2>&1
rc=$?; tail -2 gpurun_out/$TAG/smoke.log; [ $rc -ne 0 ] && exit $rc
TAG=$TAG SKIP_PMC=1 bash scripts/gpu_measure.sh
