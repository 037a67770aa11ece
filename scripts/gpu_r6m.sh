#!/bin/bash
# Round 6 (m): the GAE / normaliser tests, then the HBM legs + the off-policy legs (reuse
# configurations up to 262144 x 1) on the in-tree build; GAE stages the per-step reward
# statistics in LDS (r6fin: 45.7 us with them in registers).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); TAG=${TAG:-r6m}; OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"
( while sleep 30; do echo "[$(date +%T)] alive" >> "$OUT/progress.log"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
log() { echo "[$(date +%T)] $*" | tee -a "$OUT/progress.log"; }
stop() { log "STOP: $1 rc=$2"; exit "$2"; }
log "tests"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dppo2.py -m gpu -x -q \
    -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; tail -1 "$OUT/tests.log" | tee -a "$OUT/progress.log"; [ $rc -ne 0 ] && stop tests $rc
log "bench hbm + off-policy legs"
timeout -k 10 500 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --e2e 0 --fp32-leg 0 \
    --uav 0 --oa 0 --demo-e2e 0 > "$OUT/bench.log" 2>&1
rc=$?; tail -1 "$OUT/bench.log" > "$OUT/bench.json"; [ $rc -ne 0 ] && stop bench $rc
python3 - "$OUT/bench.json" <<'PY' | tee -a "$OUT/progress.log"
import json, sys
d = json.loads(open(sys.argv[1]).read())
print(json.dumps({k: [round(v["avg_launch_ms"] * 1e3, 2), round(v["frac"], 3)] for k, v in d.get("hbm_kernels", {}).items()}))
for leg in ("soi_ddpg", "ugvoa_sac"):
    for r in d.get(leg, {}).get("reference_reuse", []):
        print(leg, r["batch"], r["learn_iters_per_step"], round(r["value"]), round(r["learn_ms"], 3), round(r["learn_roofline"]["frac"], 3))
PY
log DONE
