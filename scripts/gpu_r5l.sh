#!/bin/bash
# Round 5: the rollout's f16 split through v_fma_mix (early-clobber form, build expR) against the
# in-tree packed-convert split: rollout parity tests on expR, then a same-box A/B of the rollout legs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${TAG:-r5l}; OUT=gpurun_out/$T; mkdir -p "$OUT"
C=reinforcementlearningplatform_amd/csrc/build
RLP_LIBRARY=$(pwd)/$C/expR/librlp.so timeout -k 10 400 python -u -m pytest tests/test_gpu_rollout.py tests/test_gpu_rollout_parity.py -x -q --timeout 120 --timeout-method thread -m gpu > "$OUT/tests_expR.log" 2>&1
rc=$?; tail -3 "$OUT/tests_expR.log"; echo "expR tests rc=$rc"
[ $rc -ne 0 ] && exit $rc
TAG=$T/ab REPS=${REPS:-3} LIBS="- $C/expR/librlp.so" ARGS="--uav 1 --steps 20 --warmup 5" PAT="rollout_sp" \
  bash scripts/gpu_lib_ab.sh
