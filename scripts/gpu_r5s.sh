#!/bin/bash
# Round 5: layer-2 weight operands of the fused gradient in registers: the demo
# nets' tests, then a same-box A/B against HEAD's rlp_dense (expB).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${TAG:-r5s}; OUT=gpurun_out/$T; mkdir -p "$OUT"
C=reinforcementlearningplatform_amd/csrc/build
timeout -k 10 400 python -u -m pytest tests/test_gpu_plain_nets.py tests/test_gpu_dropin.py -x -q --timeout 120 --timeout-method thread -m gpu > "$OUT/tests.log" 2>&1
rc=$?; tail -2 "$OUT/tests.log"; echo "tests rc=$rc"
[ $rc -ne 0 ] && exit $rc
TAG=$T/ab REPS=${REPS:-2} LIBS="- $C/expB/librlp.so" ARGS="--e2e 0 --e2e-k30 0 --demo-e2e 1" \
  PAT="fg_grad" bash scripts/gpu_lib_ab.sh
