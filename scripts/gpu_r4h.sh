#!/bin/bash
# Round-4 call h: exp4 = the two-stage dense GEMM (128-row register-prefetched stages, 67.6 KB LDS,
# two blocks per CU) + the PPO2 gradient reduce with its partial loads unrolled: the full GPU test
# suite on it, the off-policy / demo bench legs and the DDPG / SAC learn() kernel timelines under
# it (+ the fused three-layer forward chains of the DDPG nets / SAC critics), the same legs on the
# in-tree build, then an e2e A/B for the reduce.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; TAG=${TAG:-r4h}; mkdir -p "$OUT/$TAG"
export TMPDIR=/tmp
export RLP_LIBRARY=$ROOT/reinforcementlearningplatform_amd/csrc/build/exp4/librlp.so
step() { local name=$1; shift; local t0=$(date +%s); "$@" > "$OUT/$TAG/$name.log" 2>&1; local rc=$?
         echo "$name rc=$rc ($(( $(date +%s) - t0 )) s)"; tail -${TAILN:-4} "$OUT/$TAG/$name.log"; return $rc; }
step tests timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 \
     --timeout-method thread || exit $?
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/$TAG/trace" -o run \
   -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --e2e 0 --e2e-k30 0 --demo-e2e 1 \
      --uav 0 --hbm 0 --fp32-leg 0 --oa 0 --ddpg 1 --sac 1) > "$OUT/$TAG/offpolicy_bench.log" 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/dispatch_timeline.py "$OUT/$TAG/trace" ddpg_td_kernel 20 6 30 > "$OUT/$TAG/ddpg_timeline.txt" 2>&1
python3 scripts/dispatch_timeline.py "$OUT/$TAG/trace" sac_target_kernel 20 12 48 > "$OUT/$TAG/sac_timeline.txt" 2>&1
tail -1 "$OUT/$TAG/ddpg_timeline.txt"; tail -1 "$OUT/$TAG/sac_timeline.txt"
rm -rf "$OUT/$TAG/trace"
unset RLP_LIBRARY
(cd /tmp && timeout -k 10 300 python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --e2e 0 --e2e-k30 0 \
   --demo-e2e 1 --uav 0 --hbm 0 --fp32-leg 0 --oa 0 --ddpg 1 --sac 1) > "$OUT/$TAG/offpolicy_bench_base.log" 2>&1
rc=$?; echo "base bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 - "$OUT/$TAG/offpolicy_bench.log" "$OUT/$TAG/offpolicy_bench_base.log" <<'PY'
import json, sys
for f in sys.argv[1:]:
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l)
            print(f.split("/")[-1], {k: {x: d[k].get(x) for x in ("value", "learn_ms", "s_per_iteration")}
                                     for k in ("soi_ddpg", "ugvoa_sac", "soi_ppo2_e2e", "ugvoa_ppo2_e2e") if k in d})
PY
TAG=${TAG}_ab LIBS="reinforcementlearningplatform_amd/csrc/build/exp4/librlp.so -" REPS=1 \
  ARGS="--e2e 1 --e2e-k30 1 --uav 0" PAT="fd_kernel|wgrad_kernel|reduce_kernel" bash scripts/gpu_lib_ab.sh || exit $?
echo DONE
