#!/bin/bash
# Round 6 (l): the whole GPU suite + smoke on the in-tree build (lidar rollout two launches per
# step), then the rollout / UAV / HBM-legs bench, in-tree vs rlp_rollout.hip built without
# MachineLICM (fewer registers in every rollout kernel) and the UAV env step compiled for 3 / 4
# waves per SIMD (env3 / env4), alternating, two repetitions.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); TAG=${TAG:-r6l}; OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"
( while sleep 30; do echo "[$(date +%T)] alive" >> "$OUT/progress.log"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
log() { echo "[$(date +%T)] $*" | tee -a "$OUT/progress.log"; }
stop() { log "STOP: $1 rc=$2"; exit "$2"; }
NL=$ROOT/reinforcementlearningplatform_amd/csrc/build/expnolicm_ro/librlp.so
log "suite"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
    --timeout-method thread > "$OUT/suite.log" 2>&1
rc=$?; tail -1 "$OUT/suite.log" | tee -a "$OUT/progress.log"; [ $rc -ne 0 ] && stop suite $rc
log "smoke"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; tail -1 "$OUT/smoke.log" | tee -a "$OUT/progress.log"; [ $rc -ne 0 ] && stop smoke $rc
BA="--steps 10 --warmup 3 --no-cpu-baseline --e2e 0 --fp32-leg 0 --ddpg 0 --oa 0 --sac 0 --demo-e2e 0"
for rep in 1 2; do
  for lib in - nolicm env3 env4; do
    log "bench A/B rep $rep lib=$lib"
    case $lib in
      -) unset RLP_LIBRARY ;;
      nolicm) export RLP_LIBRARY=$NL ;;
      *) export RLP_LIBRARY=$ROOT/reinforcementlearningplatform_amd/csrc/build/exp$lib/librlp.so ;;
    esac
    timeout -k 10 300 python -u bench.py $BA > "$OUT/bench_$lib.log" 2>&1
    rc=$?; unset RLP_LIBRARY
    [ $rc -ne 0 ] && stop "bench $lib" $rc
    cp "$OUT/bench_$lib.log" "$OUT/bench_${lib}_$rep.log"
    python3 - "$OUT/bench_$lib.log" "$lib" <<'PY' | tee -a "$OUT/progress.log"
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        d = json.loads(line)
        o = {"lib": sys.argv[2], "value": d["value"], "frac": d["roofline"]["frac"],
             "rollout_ms": d["roofline"].get("avg_launch_ms")}
        u = d.get("uav_ppo2_rollout", {}).get("roofline", {})
        o["uav_frac"], o["uav_ms"] = u.get("frac"), u.get("avg_launch_ms")
        o["hbm"] = {k: [round(v["avg_launch_ms"] * 1e3, 2), round(v["frac"], 3)] for k, v in d.get("hbm_kernels", {}).items()}
        print(json.dumps(o))
PY
  done
done
log DONE
