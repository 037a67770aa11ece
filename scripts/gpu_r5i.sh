#!/bin/bash
# Round 5: the fused SOI-net gradient kernel and the wgrad kernel's two-step g2 prefetch: the demo
# nets' tests first (a fault stops here), then the whole GPU suite + smoke, then a same-box A/B of
# the update kernels (in-tree library against csrc/build/expB, the previous wgrad).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${TAG:-r5i}; OUT=gpurun_out/$T; mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_plain_nets.py -x -v --timeout 120 --timeout-method thread > "$OUT/plain_nets.log" 2>&1
rc=$?; grep -E "PASS|FAIL|Error|error|native err" "$OUT/plain_nets.log" | tail -30; echo "plain_nets rc=$rc"
[ $rc -ne 0 ] && exit $rc
TAG=$T bash scripts/gpu_tests.sh || exit $?
TAG=$T/ab REPS=2 LIBS="- reinforcementlearningplatform_amd/csrc/build/expB/librlp.so" \
  ARGS="--e2e 1 --e2e-k30 0 --demo-e2e 1" PAT="fd_kernel|wgrad|fg_grad|chunk_sum|loss_sum|l1_|chain|dense_gemm" \
  bash scripts/gpu_lib_ab.sh
