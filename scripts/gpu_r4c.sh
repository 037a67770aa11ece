#!/bin/bash
# Round-4 call c: GPU tests on the in-tree build, then a same-box A/B against a baseline library
# (LIBS), rocprof kernel averages + the bench's e2e / UAV numbers.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; TAG=${TAG:-r4c}; mkdir -p "$OUT/$TAG"
step() { local name=$1; shift; local t0=$(date +%s); "$@" > "$OUT/$TAG/$name.log" 2>&1; local rc=$?
         echo "$name rc=$rc ($(( $(date +%s) - t0 )) s)"; tail -${TAILN:-4} "$OUT/$TAG/$name.log"; return $rc; }
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  step tests timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 \
       --timeout-method thread ${PYTEST_ARGS:-} || exit $?
fi
TAG=${TAG}_ab LIBS="${LIBS:-reinforcementlearningplatform_amd/csrc/build/expbase/librlp.so -}" REPS=${REPS:-2} \
  ARGS="${ABARGS:---e2e 1 --e2e-k30 1 --uav 1}" PAT="${PAT:-fd_kernel|wgrad_kernel|rollout_sp}" bash scripts/gpu_lib_ab.sh || exit $?
echo DONE
