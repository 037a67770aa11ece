#!/bin/bash
# Round 5: oa_reset_kernel as a grid-stride loop (4 blocks per CU) instead of one wave per env:
# the lidar env / rollout tests, then a same-box A/B of the UGV-OA legs against HEAD's (expB).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${TAG:-r5aa}; OUT=gpurun_out/$T; mkdir -p "$OUT"
C=reinforcementlearningplatform_amd/csrc/build
timeout -k 10 400 python -u -m pytest tests/test_gpu_ugvoa.py tests/test_gpu_rollout.py -x -q --timeout 120 --timeout-method thread -m gpu > "$OUT/tests.log" 2>&1
rc=$?; tail -2 "$OUT/tests.log"; echo "tests rc=$rc"
[ $rc -ne 0 ] && exit $rc
TAG=$T/ab REPS=${REPS:-2} LIBS="- $C/expB/librlp.so" OA=1 ARGS="--e2e 0 --e2e-k30 0 --demo-e2e 1" \
  PAT="oa_reset|oa_kernel|oa_post|oa_sample" bash scripts/gpu_lib_ab.sh
