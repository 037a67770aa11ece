#!/bin/bash
# Round 5: FD kernel with 12-wave blocks (3 waves per SIMD: the backward GEMM in two output halves,
# g2 of the second half re-read from the G2 stores, dW1 partials in LDS; build expW12) against the
# 8-wave in-tree build and HEAD's (expB): the update tests on both new builds, then a same-box A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${TAG:-r5k}; OUT=gpurun_out/$T; mkdir -p "$OUT"
C=reinforcementlearningplatform_amd/csrc/build
TESTS="tests/test_gpu_update.py tests/test_learn_golden.py tests/test_gpu_plain_nets.py tests/test_gpu_dropin.py"
timeout -k 10 400 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread -m gpu > "$OUT/tests_w8.log" 2>&1
rc=$?; tail -3 "$OUT/tests_w8.log"; echo "w8 tests rc=$rc"
[ $rc -ne 0 ] && exit $rc
RLP_LIBRARY=$(pwd)/$C/expW12/librlp.so timeout -k 10 400 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread -m gpu > "$OUT/tests_w12.log" 2>&1
rc=$?; tail -3 "$OUT/tests_w12.log"; echo "w12 tests rc=$rc"
[ $rc -ne 0 ] && exit $rc
TAG=$T/ab REPS=${REPS:-2} LIBS="- $C/expW12/librlp.so $C/expB/librlp.so" \
  ARGS="--e2e 1 --e2e-k30 0 --demo-e2e 1" PAT="fd_kernel|wgrad_kernel<1" \
  bash scripts/gpu_lib_ab.sh
