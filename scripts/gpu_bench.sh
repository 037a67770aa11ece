#!/bin/bash
# The driver's bench command on the in-tree build (one JSON line into gpurun_out/$TAG/bench.json)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r5b}; mkdir -p "$OUT"
( while sleep 60; do echo "alive $(date +%T)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 900 python -u bench.py ${BENCH_ARGS:---gpus 1 --steps 20 --warmup 5} > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc"; tail -3 "$OUT/bench.err"
python3 - "$OUT/bench.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print("value %.4g  ms/step %.3f  frac %.3f  achieved %.1f TF" % (d["value"], d["ms_per_step"], r["frac"], r["achieved"]))
for k in ("uav_ppo2_rollout",):
    if k in d: print(k, "%.4g" % d[k]["value"], "frac %.3f" % d[k]["roofline"]["frac"])
e = d.get("e2e", {})
if e: print("e2e K=6 %.4f s" % e["s_per_iteration"], "K=30 %.4f s" % e.get("k30", {}).get("s_per_iteration", float("nan")),
            "upd frac k30 %.3f" % e.get("k30", {}).get("update_roofline", {}).get("frac", float("nan")))
for k in ("soi_ppo2_e2e", "ugvoa_ppo2_e2e"):
    if k in d: print(k, "%.4f s/it" % d[k]["s_per_iteration"], "update %.1f ms" % d[k]["update_ms"], "frac %.3f" % d[k]["update_roofline"]["frac"], d[k]["update"])
for k in ("soi_ddpg", "ugvoa_sac"):
    if k in d: print(k, "%.4g" % d[k]["value"], "learn %.3f ms" % d[k]["learn_ms"], "frac %.3f" % d[k]["learn_roofline"]["frac"])
if "ugvoa_ppo2_rollout" in d: print("ugvoa rollout %.4g" % d["ugvoa_ppo2_rollout"]["value"], "frac %.3f" % d["ugvoa_ppo2_rollout"]["roofline"]["frac"])
if "cpu_baseline" in d: print("cpu", d["cpu_baseline"])
PY
exit $rc
