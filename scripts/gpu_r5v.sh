#!/bin/bash
# Round 5: ppo2_fd32_kernel scheduling variants — DMA pieces spread over the chunk's MFMAs (expS1V0),
# that plus 4 VALU slots pinned after each MFMA triple (expS1V4), the bunched DMA (expF32) — against
# the in-tree 16-row FD: update tests on expS1V4, then a same-box A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${TAG:-r5v}; OUT=gpurun_out/$T; mkdir -p "$OUT"
C=reinforcementlearningplatform_amd/csrc/build
RLP_LIBRARY=$(pwd)/$C/expS1V4/librlp.so timeout -k 10 300 python -u -m pytest tests/test_gpu_update.py tests/test_learn_golden.py -x -q --timeout 120 --timeout-method thread -m gpu > "$OUT/tests.log" 2>&1
rc=$?; tail -2 "$OUT/tests.log"; echo "tests rc=$rc"
[ $rc -ne 0 ] && exit $rc
TAG=$T/ab REPS=${REPS:-2} LIBS="- $C/expF32/librlp.so $C/expS1V0/librlp.so $C/expS1V4/librlp.so" \
  ARGS="--e2e 1 --e2e-k30 0 --demo-e2e 0" PAT="fd_kernel|fd32_kernel" bash scripts/gpu_lib_ab.sh
