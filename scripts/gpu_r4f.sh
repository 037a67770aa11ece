#!/bin/bash
# Round-4 call f: the one-wave-per-SIMD FD kernel (expfd1: 4-wave blocks, the previous tile's
# g1 / dW1 tail among the next forward GEMM's MFMAs) — its update parity tests, then a same-box
# A/B against the in-tree build (8-wave FD) and expbase.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; TAG=${TAG:-r4f}; mkdir -p "$OUT/$TAG"
export TMPDIR=/tmp
step() { local name=$1; shift; local t0=$(date +%s); "$@" > "$OUT/$TAG/$name.log" 2>&1; local rc=$?
         echo "$name rc=$rc ($(( $(date +%s) - t0 )) s)"; tail -${TAILN:-4} "$OUT/$TAG/$name.log"; return $rc; }
RLP_LIBRARY=$ROOT/reinforcementlearningplatform_amd/csrc/build/expfd1/librlp.so step tests_fd1 timeout -k 10 600 \
     python -u -m pytest tests/test_gpu_update.py tests/test_learn_golden.py tests/test_gpu_dppo2.py \
     tests/test_gpu_rccl.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread || exit $?
TAG=${TAG}_ab LIBS="reinforcementlearningplatform_amd/csrc/build/expfd1/librlp.so - reinforcementlearningplatform_amd/csrc/build/expbase/librlp.so" REPS=2 \
  ARGS="--e2e 1 --e2e-k30 1 --uav 0" PAT="fd_kernel|wgrad_kernel" bash scripts/gpu_lib_ab.sh || exit $?
step tests_offpolicy timeout -k 10 600 python -u -m pytest tests/test_gpu_replay_ddpg.py tests/test_gpu_sac.py \
     tests/test_gpu_ugvoa.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread || exit $?
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/$TAG/trace" -o run \
   -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --e2e 0 --e2e-k30 0 --demo-e2e 0 \
      --uav 0 --hbm 0 --fp32-leg 0 --oa 0 --ddpg 1 --sac 1) > "$OUT/$TAG/offpolicy_bench.log" 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/dispatch_timeline.py "$OUT/$TAG/trace" ddpg_td_kernel 20 6 40 > "$OUT/$TAG/ddpg_timeline.txt" 2>&1
python3 scripts/dispatch_timeline.py "$OUT/$TAG/trace" sac_target_kernel 20 12 60 > "$OUT/$TAG/sac_timeline.txt" 2>&1
tail -1 "$OUT/$TAG/ddpg_timeline.txt"; tail -1 "$OUT/$TAG/sac_timeline.txt"
python3 - "$OUT/$TAG/offpolicy_bench.log" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l)
        for k in ("soi_ddpg", "ugvoa_sac"):
            if k in d: print(k, {x: d[k].get(x) for x in ("value", "env_only", "learn_ms")})
PY
rm -rf "$OUT/$TAG/trace"
echo DONE
