#!/bin/bash
# Round 5: ppo2_wgrad_kernel's h1 fragment builds of a SIMD's two waves staggered by half a spacing
# (expST) against the in-tree ones in step: update tests on expST, then a same-box A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${TAG:-r5y}; OUT=gpurun_out/$T; mkdir -p "$OUT"
C=reinforcementlearningplatform_amd/csrc/build
RLP_LIBRARY=$(pwd)/$C/expST/librlp.so timeout -k 10 300 python -u -m pytest tests/test_gpu_update.py tests/test_learn_golden.py -x -q --timeout 120 --timeout-method thread -m gpu > "$OUT/tests.log" 2>&1
rc=$?; tail -2 "$OUT/tests.log"; echo "tests rc=$rc"
[ $rc -ne 0 ] && exit $rc
TAG=$T/ab REPS=${REPS:-2} LIBS="- $C/expST/librlp.so" \
  ARGS="--e2e 1 --e2e-k30 0 --demo-e2e 1" PAT="wgrad_kernel" bash scripts/gpu_lib_ab.sh
