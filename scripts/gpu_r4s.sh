#!/bin/bash
# Round-4 closing check: the GPU suite and smoke on the in-tree build at HEAD (no variant library).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r4s}; mkdir -p gpurun_out/$TAG
unset RLP_LIBRARY
timeout -k 10 600 python -u -m pytest -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider tests > gpurun_out/$TAG/tests.log 2>&1
rc=$?; tail -3 gpurun_out/$TAG/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/$TAG/smoke.log 2>&1
rc=$?; tail -2 gpurun_out/$TAG/smoke.log; exit $rc
