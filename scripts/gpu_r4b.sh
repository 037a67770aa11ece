#!/bin/bash
# Round-4 call b: the new gradient-pin tests, then the in-training rollout diagnosis
# (scripts/diag_e2e_rollout.py plain, then under a GRBM_GUI_ACTIVE / L2 counter pass).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; TAG=${TAG:-r4b}; mkdir -p "$OUT/$TAG"
export TMPDIR=/tmp
step() { local name=$1; shift; local t0=$(date +%s); "$@" > "$OUT/$TAG/$name.log" 2>&1; local rc=$?
         echo "$name rc=$rc ($(( $(date +%s) - t0 )) s)"; tail -${TAILN:-6} "$OUT/$TAG/$name.log"; return $rc; }
step tests timeout -k 10 600 python -u -m pytest -p no:cacheprovider --timeout 200 --timeout-method thread -q -s \
     tests/test_offpolicy_grad_golden.py tests/test_gpu_sac.py tests/test_gpu_replay_ddpg.py -m gpu || exit $?
TAILN=12 step diag timeout -k 10 300 python -u scripts/diag_e2e_rollout.py || exit $?
(cd /tmp && timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv \
   -d "$OUT/$TAG/pmc1" -o run -- python3 "$ROOT/scripts/diag_e2e_rollout.py") > "$OUT/$TAG/pmc1.log" 2>&1
rc=$?; echo "pmc1 rc=$rc"; tail -8 "$OUT/$TAG/pmc1.log"; [ $rc -ne 0 ] && exit $rc
python3 scripts/pmc_dispatches.py "$OUT/$TAG/pmc1" rollout_sp_kernel > "$OUT/$TAG/pmc1_dispatches.txt"; cat "$OUT/$TAG/pmc1_dispatches.txt"
(cd /tmp && timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv \
   -d "$OUT/$TAG/pmc2" -o run -- python3 "$ROOT/scripts/diag_e2e_rollout.py") > "$OUT/$TAG/pmc2.log" 2>&1
rc=$?; echo "pmc2 rc=$rc"; tail -3 "$OUT/$TAG/pmc2.log"; [ $rc -ne 0 ] && exit $rc
python3 scripts/pmc_dispatches.py "$OUT/$TAG/pmc2" rollout_sp_kernel > "$OUT/$TAG/pmc2_dispatches.txt"; cat "$OUT/$TAG/pmc2_dispatches.txt"
RLP_LIBRARY=$ROOT/reinforcementlearningplatform_amd/csrc/build/exprot/librlp.so step rot_tests timeout -k 10 600 \
     python -u -m pytest -p no:cacheprovider --timeout 200 --timeout-method thread -q tests/test_learn_golden.py \
     tests/test_gpu_update.py tests/test_gpu_dppo2.py -m gpu || exit $?
TAG=r4b_ab LIBS="- reinforcementlearningplatform_amd/csrc/build/exprot/librlp.so" REPS=2 ARGS="--e2e 1 --e2e-k30 1" \
  PAT="fd_kernel|wgrad_kernel|rollout_sp" bash scripts/gpu_lib_ab.sh || exit $?
echo DONE
