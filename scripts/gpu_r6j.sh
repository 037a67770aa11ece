#!/bin/bash
# Round 6 (j): the lidar one-launch segment kernel built without MachineLICM (no scratch: the
# hoisted loop invariants were what spilled), after the context that faulted it (the two-thread
# per-call test), then the whole suite on that build; the lidar leg; rollout / HBM bench legs
# in-tree vs that build (A/B, alternating). Progress to gpurun_out/$TAG/progress.log.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); TAG=${TAG:-r6j}; OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"
( while sleep 30; do echo "[$(date +%T)] alive" >> "$OUT/progress.log"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
log() { echo "[$(date +%T)] $*" | tee -a "$OUT/progress.log"; }
stop() { log "STOP: $1 rc=$2"; exit "$2"; }
NL=$ROOT/reinforcementlearningplatform_amd/csrc/build/expnolicm_ro/librlp.so
PYT="python -u -m pytest -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread"
log "ctx repro on no-LICM build, one launch"
RLP_LIBRARY=$NL RLP_OA_ONE_LAUNCH=1 timeout -k 10 300 $PYT \
    tests/test_gpu_rollout.py::test_two_threads_choose_precision_per_call \
    tests/test_gpu_rollout_parity.py::test_rollout_lidar_env_teacher_forced_config5_shard > "$OUT/ctx.log" 2>&1
rc=$?; tail -2 "$OUT/ctx.log" | tee -a "$OUT/progress.log"; [ $rc -ne 0 ] && stop ctx $rc
log "suite on no-LICM build, one launch"
RLP_LIBRARY=$NL RLP_OA_ONE_LAUNCH=1 timeout -k 10 900 $PYT tests > "$OUT/suite.log" 2>&1
rc=$?; tail -2 "$OUT/suite.log" | tee -a "$OUT/progress.log"; [ $rc -ne 0 ] && stop suite $rc
for rep in 1 2; do
  log "lidar leg no-LICM one launch rep $rep"
  RLP_LIBRARY=$NL RLP_OA_ONE_LAUNCH=1 timeout -k 10 300 python -u scripts/leg.py ugvoa_ppo2_leg > "$OUT/leg.log" 2>&1
  rc=$?; tail -1 "$OUT/leg.log" >> "$OUT/legs.jsonl"; tail -1 "$OUT/leg.log" | cut -c1-200 | tee -a "$OUT/progress.log"
  [ $rc -ne 0 ] && stop leg $rc
done
BA="--steps 10 --warmup 3 --no-cpu-baseline --e2e 0 --fp32-leg 0 --ddpg 0 --oa 0 --sac 0 --demo-e2e 0"
for rep in 1 2; do
  for lib in - nolicm; do
    log "bench A/B rep $rep lib=$lib"
    if [ "$lib" = - ]; then unset RLP_LIBRARY; else export RLP_LIBRARY=$NL; fi
    timeout -k 10 300 python -u bench.py $BA > "$OUT/bench_$lib.log" 2>&1
    rc=$?; unset RLP_LIBRARY
    [ $rc -ne 0 ] && stop "bench $lib" $rc
    python3 - "$OUT/bench_$lib.log" "$lib" <<'PY' | tee -a "$OUT/progress.log"
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        d = json.loads(line)
        o = {"lib": sys.argv[2], "value": d["value"], "ms": d["ms_per_step"], "frac": d["roofline"]["frac"],
             "rollout_ms": d["roofline"].get("avg_launch_ms")}
        u = d.get("uav_ppo2_rollout", {}).get("roofline", {})
        o["uav_frac"], o["uav_ms"] = u.get("frac"), u.get("avg_launch_ms")
        for k, v in d.get("hbm_kernels", {}).items():
            o[k] = round(v["avg_launch_ms"] * 1e3, 2)
        print(json.dumps(o))
PY
  done
done
log DONE
