#!/bin/bash
# Round 5: FD / wgrad VALU trims (early-clobber f16 split, broadcast b1 from LDS): the update tests,
# then a same-box A/B against HEAD's update (expB) and two timing-only diagnostics of the FD kernel
# (no W2 chunk DMA after the first tile; that and no ring barriers: wrong gradients, timing only).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${TAG:-r5j}; OUT=gpurun_out/$T; mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_update.py tests/test_learn_golden.py tests/test_gpu_plain_nets.py -x -q --timeout 120 --timeout-method thread -m gpu > "$OUT/update_tests.log" 2>&1
rc=$?; tail -5 "$OUT/update_tests.log"; echo "update tests rc=$rc"
[ $rc -ne 0 ] && exit $rc
C=reinforcementlearningplatform_amd/csrc/build
TAG=$T/ab REPS=${REPS:-2} LIBS="- $C/expB/librlp.so $C/exp_nodma/librlp.so $C/exp_nodma_nobar/librlp.so" \
  ARGS="--e2e 1 --e2e-k30 0 --demo-e2e 0" PAT="fd_kernel<1|wgrad_kernel<1" \
  bash scripts/gpu_lib_ab.sh
