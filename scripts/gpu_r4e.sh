#!/bin/bash
# Round-4 call e: GPU tests on the in-tree build (FD: dW1 back on VALU, the g1 tail's layer-1
# MFMAs batched, the actor loss inputs prefetched), a same-box FD A/B against expbase, and the
# kernel timeline of one DDPG / SAC learn() inside the bench's captured HIP graphs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; TAG=${TAG:-r4e}; mkdir -p "$OUT/$TAG"
export TMPDIR=/tmp
step() { local name=$1; shift; local t0=$(date +%s); "$@" > "$OUT/$TAG/$name.log" 2>&1; local rc=$?
         echo "$name rc=$rc ($(( $(date +%s) - t0 )) s)"; tail -${TAILN:-4} "$OUT/$TAG/$name.log"; return $rc; }
step tests timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 \
     --timeout-method thread || exit $?
TAG=${TAG}_ab LIBS="reinforcementlearningplatform_amd/csrc/build/expbase/librlp.so -" REPS=2 \
  ARGS="--e2e 1 --e2e-k30 1 --uav 0" PAT="fd_kernel|wgrad_kernel" bash scripts/gpu_lib_ab.sh || exit $?
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/$TAG/trace" -o run \
   -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --e2e 0 --e2e-k30 0 --demo-e2e 0 \
      --uav 0 --hbm 0 --fp32-leg 0 --oa 0 --ddpg 1 --sac 1) > "$OUT/$TAG/offpolicy_bench.log" 2>&1
rc=$?; echo "trace rc=$rc"; tail -2 "$OUT/$TAG/offpolicy_bench.log" | cut -c1-300; [ $rc -eq 0 ] || exit $rc
python3 scripts/dispatch_timeline.py "$OUT/$TAG/trace" ddpg_td_kernel 20 6 40 > "$OUT/$TAG/ddpg_timeline.txt" 2>&1
python3 scripts/dispatch_timeline.py "$OUT/$TAG/trace" sac_target_kernel 20 12 60 > "$OUT/$TAG/sac_timeline.txt" 2>&1
tail -3 "$OUT/$TAG/ddpg_timeline.txt"; tail -3 "$OUT/$TAG/sac_timeline.txt"
rm -rf "$OUT/$TAG/trace"
echo DONE
