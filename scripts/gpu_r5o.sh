#!/bin/bash
# Round 5: FD ring shapes — 2 chunks per ring slot (one barrier per phase: expC2), a 4-slot ring
# (expR4), both (expC2R4) — against the in-tree 3 x 1 ring: the update tests on each build, then a
# same-box A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${TAG:-r5o}; OUT=gpurun_out/$T; mkdir -p "$OUT"
C=reinforcementlearningplatform_amd/csrc/build
TESTS="tests/test_gpu_update.py tests/test_learn_golden.py tests/test_gpu_plain_nets.py"
for v in C2 R4 C2R4; do
  RLP_LIBRARY=$(pwd)/$C/exp$v/librlp.so timeout -k 10 300 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread -m gpu > "$OUT/tests_$v.log" 2>&1
  rc=$?; tail -1 "$OUT/tests_$v.log"; echo "$v tests rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
TAG=$T/ab REPS=${REPS:-2} LIBS="- $C/expC2/librlp.so $C/expR4/librlp.so $C/expC2R4/librlp.so" \
  ARGS="--e2e 1 --e2e-k30 0 --demo-e2e 1" PAT="fd_kernel" \
  bash scripts/gpu_lib_ab.sh
