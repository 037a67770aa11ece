#!/bin/bash
# Round-4 call l: the full GPU suite on exp10 (exp9 + eight-wave chains), then the off-policy /
# demo legs on exp7 (chains, SAC actor chain), exp8 (+ the actors' batched-inference chain),
# exp9 (+ multi-problem GEMM launches and the weight-gradient chains) and exp10, and exp10's
# learn() timelines. Call n: V=exp12 AB="base exp11 exp12" (exp11: two 16-row tiles per forward
# block for batched inference; exp12: + the SAC actor's backward as one data chain + one launch).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; TAG=${TAG:-r4l}; mkdir -p "$OUT/$TAG"
# call o was queued for exp14 (hoisted weight loads) before exp15 (+ the PPO2 dense forward and the
# tanh nets' inference as chains) was built: it runs the superset
if [ "$TAG" = r4o ]; then V=exp15; AB="base exp14 exp15"; fi
export TMPDIR=/tmp
LIBD=reinforcementlearningplatform_amd/csrc/build
export RLP_LIBRARY=$ROOT/$LIBD/${V:-exp10}/librlp.so
timeout -k 10 700 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 200 \
   --timeout-method thread > "$OUT/$TAG/tests.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -12 "$OUT/$TAG/tests.log"
case $rc in 0|1) ;; *) exit $rc;; esac
LEGS="--steps 3 --warmup 1 --no-cpu-baseline --e2e 0 --e2e-k30 0 --demo-e2e 1 --uav 0 --hbm 0 --fp32-leg 0 --oa 0 --ddpg 1 --sac 1"
for v in ${AB:-exp7 exp8 exp9 exp10}; do
  if [ $v = base ]; then unset RLP_LIBRARY; else export RLP_LIBRARY=$ROOT/$LIBD/$v/librlp.so; fi
  (cd /tmp && timeout -k 10 300 python3 "$ROOT/bench.py" $LEGS) > "$OUT/$TAG/bench_$v.log" 2>&1
  rc=$?; echo "bench $v rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 - "$OUT/$TAG" ${AB:-exp7 exp8 exp9 exp10} <<'PY'
import json, sys
for v in sys.argv[2:]:
    for l in open(f"{sys.argv[1]}/bench_{v}.log"):
        if l.startswith("{"):
            d = json.loads(l)
            print(v, {k: {x: round(d[k][x], 4) if isinstance(d[k].get(x), float) and x != "value" else d[k].get(x)
                          for x in ("value", "learn_ms", "s_per_iteration")}
                      for k in ("soi_ddpg", "ugvoa_sac", "soi_ppo2_e2e", "ugvoa_ppo2_e2e") if k in d})
PY
export RLP_LIBRARY=$ROOT/$LIBD/${V:-exp10}/librlp.so
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/$TAG/trace" -o run \
   -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --e2e 0 --e2e-k30 0 --demo-e2e 0 \
      --uav 0 --hbm 0 --fp32-leg 0 --oa 0 --ddpg 1 --sac 1) > "$OUT/$TAG/trace_bench.log" 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/dispatch_timeline.py "$OUT/$TAG/trace" ddpg_td_kernel 20 6 30 > "$OUT/$TAG/ddpg_timeline.txt" 2>&1
python3 scripts/dispatch_timeline.py "$OUT/$TAG/trace" sac_target_kernel 20 12 48 > "$OUT/$TAG/sac_timeline.txt" 2>&1
tail -1 "$OUT/$TAG/ddpg_timeline.txt"; tail -1 "$OUT/$TAG/sac_timeline.txt"
rm -rf "$OUT/$TAG/trace"
echo DONE
