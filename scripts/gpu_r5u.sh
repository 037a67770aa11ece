#!/bin/bash
# Round 5: ppo2_fd32_kernel (32-row waves on v_mfma_f32_32x32x16_f16, one wave per SIMD; build
# expF32): the update tests on it (a fault stops here), then a same-box A/B against the in-tree FD.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${TAG:-r5u}; OUT=gpurun_out/$T; mkdir -p "$OUT"
C=reinforcementlearningplatform_amd/csrc/build
RLP_LIBRARY=$(pwd)/$C/expF32/librlp.so timeout -k 10 300 python -u -m pytest tests/test_gpu_update.py tests/test_learn_golden.py -x -v --timeout 120 --timeout-method thread -m gpu > "$OUT/tests_f32.log" 2>&1
rc=$?; grep -E "PASS|FAIL|rror" "$OUT/tests_f32.log" | tail -30; echo "fd32 tests rc=$rc"
[ $rc -ne 0 ] && exit $rc
TAG=$T/ab REPS=${REPS:-2} LIBS="- $C/expF32/librlp.so" ARGS="--e2e 1 --e2e-k30 0 --demo-e2e 0" \
  PAT="fd_kernel|fd32_kernel|wgrad_kernel<1" bash scripts/gpu_lib_ab.sh
