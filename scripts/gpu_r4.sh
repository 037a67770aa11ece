#!/bin/bash
# Round-4 GPU call: GPU tests, smoke, the driver's bench line at N=1, and an N=2 rehearsal of the
# self-launching bench (gloo, both ranks on the one GPU) plus the clear refusal of --gpus 2 over
# RCCL on a 1-GPU box. Every GPU step has its own limit; the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; TAG=${TAG:-r4a}; mkdir -p "$OUT/$TAG"
step() { local name=$1; shift; local t0=$(date +%s); "$@" > "$OUT/$TAG/$name.log" 2>&1; local rc=$?
         echo "$name rc=$rc ($(( $(date +%s) - t0 )) s)"; tail -4 "$OUT/$TAG/$name.log"; return $rc; }
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  step tests timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 \
       --timeout-method thread ${PYTEST_ARGS:-} || exit $?
  step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
fi
if [ "${SKIP_BENCH:-0}" != 1 ]; then
  step bench timeout -k 10 600 python bench.py ${BENCH_ARGS:---gpus 1 --steps 20 --warmup 5} || exit $?
fi
if [ "${SKIP_N2:-0}" != 1 ]; then
  step n2_refuse timeout -k 10 120 python bench.py --gpus 2 --steps 2 --warmup 1
  [ $? -eq 1 ] || { echo "expected the clear refusal (exit 1)"; exit 3; }
  RLP_BENCH_BACKEND=gloo step n2_gloo timeout -k 10 600 python bench.py --gpus 2 --steps 5 --warmup 2 \
       --no-cpu-baseline --ddpg 0 --oa 0 --sac 0 --hbm 0 --fp32-leg 0 --e2e 2 || exit $?
fi
echo DONE
