#!/bin/bash
# One gpurun call: the full GPU test suite and smoke at HEAD, then a same-box library A/B
# (scripts/gpu_lib_ab.sh with the caller's LIBS / ARGS / PAT / REPS). Each GPU step is time-limited
# and a failure stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${TAG:-r3z}; mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests > gpurun_out/$T/tests.log 2>&1
rc=$?; tail -3 gpurun_out/$T/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/$T/smoke.log 2>&1
rc=$?; tail -2 gpurun_out/$T/smoke.log; [ $rc -ne 0 ] && exit $rc
TAG=$T/ab bash scripts/gpu_lib_ab.sh
rc=$?; [ $rc -ne 0 ] && exit $rc
# optional: parity tests of a variant library (VARIANT_TESTS with RLP_LIBRARY=VARIANT_LIB)
if [ -n "${VARIANT_LIB:-}" ]; then
  RLP_LIBRARY=$(pwd)/$VARIANT_LIB timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread \
      -p no:cacheprovider ${VARIANT_TESTS:-tests} > gpurun_out/$T/variant_tests.log 2>&1
  rc=$?; echo "variant tests ($VARIANT_LIB):"; tail -3 gpurun_out/$T/variant_tests.log; exit $rc
fi
