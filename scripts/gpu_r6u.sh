#!/bin/bash
# Round 6 (u): GAE with the next chunk's loads issued before the current chunk's recurrence
# (build/expgaepipe): the GAE / normaliser parity tests on that build, then the HBM legs in-tree vs
# that build, alternating, two repetitions.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); TAG=${TAG:-r6u}; OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"
( while sleep 30; do echo "[$(date +%T)] alive" >> "$OUT/progress.log"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
log() { echo "[$(date +%T)] $*" | tee -a "$OUT/progress.log"; }
stop() { log "STOP: $1 rc=$2"; exit "$2"; }
GP=$ROOT/reinforcementlearningplatform_amd/csrc/build/expgaepipe/librlp.so
log "tests on the pipelined-GAE build"
RLP_LIBRARY=$GP timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dppo2.py -m gpu -x -q \
    -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; tail -1 "$OUT/tests.log" | tee -a "$OUT/progress.log"; [ $rc -ne 0 ] && stop tests $rc
BA="--steps 3 --warmup 1 --no-cpu-baseline --e2e 0 --fp32-leg 0 --uav 0 --ddpg 0 --oa 0 --sac 0 --demo-e2e 0"
for rep in 1 2; do
  for lib in - gaepipe; do
    log "bench hbm legs rep $rep lib=$lib"
    if [ "$lib" = - ]; then unset RLP_LIBRARY; else export RLP_LIBRARY=$GP; fi
    timeout -k 10 300 python -u bench.py $BA > "$OUT/bench.log" 2>&1
    rc=$?; unset RLP_LIBRARY; [ $rc -ne 0 ] && stop "bench $lib" $rc
    python3 - "$OUT/bench.log" "$lib" <<'PY' | tee -a "$OUT/progress.log"
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        d = json.loads(line)
        print(json.dumps({"lib": sys.argv[2], "hbm": {k: [round(v["avg_launch_ms"] * 1e3, 2), round(v["frac"], 3)] for k, v in d.get("hbm_kernels", {}).items()}}))
PY
  done
done
log DONE
