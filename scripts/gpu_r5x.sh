#!/bin/bash
# Round 5: ppo2_wgrad_kernel's h1 fragment builds grouped — 2 fragments per build point (expG2),
# all 4 at one point (expG4) — against the in-tree one per point: update tests on expG4, A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${TAG:-r5x}; OUT=gpurun_out/$T; mkdir -p "$OUT"
C=reinforcementlearningplatform_amd/csrc/build
RLP_LIBRARY=$(pwd)/$C/expG4/librlp.so timeout -k 10 300 python -u -m pytest tests/test_gpu_update.py tests/test_learn_golden.py -x -q --timeout 120 --timeout-method thread -m gpu > "$OUT/tests.log" 2>&1
rc=$?; tail -2 "$OUT/tests.log"; echo "tests rc=$rc"
[ $rc -ne 0 ] && exit $rc
TAG=$T/ab REPS=${REPS:-2} LIBS="- $C/expG2/librlp.so $C/expG4/librlp.so" \
  ARGS="--e2e 1 --e2e-k30 0 --demo-e2e 1" PAT="wgrad_kernel" bash scripts/gpu_lib_ab.sh
