#!/bin/bash
# One gpurun call: the full GPU test suite, smoke, then same-box A/B benches of the scheduling
# knobs (rollout / update young-half priority, FD block shape) and the off-policy legs. Each GPU
# step has its own time limit; a crash or timeout stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r3n}; mkdir -p "$OUT"
stop() { rc=$1; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "STOP rc=$rc at $2"; exit "$rc"; fi; }
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests > "$OUT/tests.log" 2>&1
  rc=$?; tail -3 "$OUT/tests.log"; stop $rc tests
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
  rc=$?; tail -1 "$OUT/smoke.log"; stop $rc smoke
fi
R="--no-cpu-baseline --ddpg 0 --sac 0 --oa 0 --fp32-leg 0 --hbm 0"
i=0
while IFS= read -r b; do
  [ -z "$b" ] && continue
  i=$((i+1))
  timeout -k 10 300 python bench.py $b > "$OUT/ab$i.log" 2>&1 < /dev/null
  rc=$?; echo "ab $i ($b) rc=$rc"; stop $rc "ab$i"
  python - "$OUT/ab$i.log" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        d = json.loads(line)
        out = {"ms": round(d["roofline"]["avg_launch_ms"], 4), "frac": round(d["roofline"]["frac"], 4)}
        if "uav_ppo2_rollout" in d: out["uav_ms"] = round(d["uav_ppo2_rollout"]["roofline"]["avg_launch_ms"], 4)
        if "e2e" in d:
            out["e2e_k6"] = round(d["e2e"]["s_per_iteration"], 4)
            if "k30" in d["e2e"]: out["e2e_k30"] = round(d["e2e"]["k30"]["s_per_iteration"], 4)
        for k in ("soi_ddpg", "ugvoa_sac", "ugvoa_ppo2_rollout", "ugvoa_lidar"):
            if k in d: out[k] = {kk: d[k][kk] for kk in ("value", "learn_ms", "with_learn_torch_update", "ms_per_segment") if kk in d[k]}
        print(json.dumps(out))
PY
done <<BENCHES
--steps 20 --warmup 5 $R --e2e 0 --uav 1 --rollout-prio 0
--steps 20 --warmup 5 $R --e2e 0 --uav 1 --rollout-prio 1
--steps 3 --warmup 1 $R --uav 0 --e2e 1 --e2e-k30 1 --update-prio 0 --fd-mode 0
--steps 3 --warmup 1 $R --uav 0 --e2e 1 --e2e-k30 1 --update-prio 1 --fd-mode 0
--steps 3 --warmup 1 $R --uav 0 --e2e 1 --e2e-k30 1 --update-prio 1 --fd-mode 1
--steps 3 --warmup 1 $R --uav 0 --e2e 1 --e2e-k30 1 --update-prio 0 --fd-mode 1
--steps 20 --warmup 5 $R --e2e 0 --uav 1 --rollout-prio 0
--steps 3 --warmup 1 --no-cpu-baseline --fp32-leg 0 --hbm 0 --uav 0 --e2e 0 --ddpg 1 --sac 1 --oa 1
BENCHES
echo DONE
