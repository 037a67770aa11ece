#!/bin/bash
# Round-4 call d: dense-grad diagnostic over batch sizes, GPU tests on the in-tree build, then a
# same-box A/B: expbase (FD dW1 on VALU) / expc (dW1 on MFMA, commit 4f2e6d8) / in-tree (+ g2 in
# the backward operand build with a bound-based scale, loss inputs prefetched, G2 stores at the
# tile end; fused reduce + Adam + soft update in the DDPG / SAC updates).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; TAG=${TAG:-r4d}; mkdir -p "$OUT/$TAG"
step() { local name=$1; shift; local t0=$(date +%s); "$@" > "$OUT/$TAG/$name.log" 2>&1; local rc=$?
         echo "$name rc=$rc ($(( $(date +%s) - t0 )) s)"; tail -${TAILN:-4} "$OUT/$TAG/$name.log"; return $rc; }
TAILN=30 step diag timeout -k 10 300 python -u scripts/diag_dense_grad.py soi || exit $?
step tests timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 \
     --timeout-method thread || exit $?
RLP_LIBRARY=$ROOT/reinforcementlearningplatform_amd/csrc/build/expc/librlp.so step offpolicy_c timeout -k 10 300 python -u scripts/ddpg_prof.py 30 4096 both || exit $?
step offpolicy_new timeout -k 10 300 python -u scripts/ddpg_prof.py 30 4096 both || exit $?
TAG=${TAG}_ab LIBS="reinforcementlearningplatform_amd/csrc/build/expbase/librlp.so reinforcementlearningplatform_amd/csrc/build/expc/librlp.so -" REPS=2 \
  ARGS="--e2e 1 --e2e-k30 1 --uav 1" PAT="fd_kernel|wgrad_kernel|rollout_sp" bash scripts/gpu_lib_ab.sh || exit $?
echo DONE
