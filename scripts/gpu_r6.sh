#!/bin/bash
# Round-6 GPU call: every step appends to gpurun_out/$TAG/progress.log (a file under gpurun_out/
# is what gpurun's silence check watches, and it survives a kill), a heartbeat appends to the same
# file every 30 s, and each GPU step runs under its own time limit; the first failing step ends the
# call (no retries). Steps, all optional, in this order:
#   TESTS="<pytest args>"     pytest -m gpu over these (default: none; "all" = the whole GPU suite)
#   SMOKE=1                   __graft_entry__.smoke()
#   LEGS="leg[:k=v,...] ..."  scripts/leg.py runs (bench legs by name), JSON lines to legs.jsonl
#   TRACE_LEGS="..."          the same legs under rocprofv3 --kernel-trace --stats (summary kept)
#   LEG_AB="leg[:k=v]" LIBS="- path ..." [REPS=n]   the leg once per library ("-" = in-tree;
#                             RLP_LIBRARY=<path> otherwise), alternating, REPS rounds
#   FD_AB=1 LIBS=...          bench.py --e2e 1 --e2e-k30 1 (rollout legs off) per library under the
#                             kernel trace: FD / wgrad averages and the e2e iteration times
#   BENCH="<bench args>"      python bench.py <args> (the JSON line to bench.json)
#   BENCH_TRACE="<args>"      bench.py <args> under rocprofv3 --kernel-trace --stats
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); TAG=${TAG:-r6}; OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
log() { echo "[$(date +%T)] $*" | tee -a "$OUT/progress.log"; }
( while sleep 30; do echo "[$(date +%T)] alive" >> "$OUT/progress.log"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
step_rc() {  # rc, what: stop the call on any failure
  if [ "$1" -ne 0 ]; then log "STOP: $2 rc=$1"; exit "$1"; fi
}
kstats() {  # summarise a rocprofv3 stats csv: librlp kernels, calls, avg us
  python3 - "$1" <<'PY'
import csv, glob, sys
fs = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)
for f in fs:
    rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))
    for r in rows[:40]:
        print("%-96s %6s %10.1f us %9.2f ms" % (r["Name"][:96], r["Calls"], float(r["AverageNs"]) / 1e3,
                                               float(r["TotalDurationNs"]) / 1e6))
PY
}
if [ -n "${TESTS:-}" ]; then
  [ "$TESTS" = all ] && TESTS=tests
  log "pytest $TESTS"
  timeout -k 10 1000 python -u -m pytest $TESTS -m gpu -x -q -p no:cacheprovider --timeout 300 \
      --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
  rc=$?; tail -25 "$OUT/gpu_tests.log" | tee -a "$OUT/progress.log"; step_rc $rc pytest
fi
if [ "${SMOKE:-0}" = 1 ]; then
  log "smoke"
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
  rc=$?; tail -3 "$OUT/smoke.log" | tee -a "$OUT/progress.log"; step_rc $rc smoke
fi
run_leg() {  # "name:k=v,k=v" -> python scripts/leg.py name k=v k=v
  local spec=$1 name args
  name=${spec%%:*}; args=""
  [ "$spec" != "$name" ] && args=$(echo "${spec#*:}" | tr ',' ' ')
  echo "$name $args"
}
for spec in ${LEGS:-}; do
  set -- $(run_leg "$spec")
  log "leg $*"
  timeout -k 10 300 python -u scripts/leg.py "$@" > "$OUT/leg.log" 2>&1
  rc=$?; tail -1 "$OUT/leg.log" >> "$OUT/legs.jsonl"; tail -c 1500 "$OUT/leg.log" | tee -a "$OUT/progress.log"
  step_rc $rc "leg $spec"
done
i=0
for spec in ${TRACE_LEGS:-}; do
  i=$((i+1)); set -- $(run_leg "$spec")
  log "traced leg $*"
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/tl$i" -o run \
      -- python3 "$ROOT/scripts/leg.py" "$@") > "$OUT/tl$i.log" 2>&1
  rc=$?; tail -1 "$OUT/tl$i.log" >> "$OUT/legs_traced.jsonl"; step_rc $rc "traced leg $spec"
  kstats "$OUT/tl$i" > "$OUT/tl${i}_stats.txt"; head -25 "$OUT/tl${i}_stats.txt" | tee -a "$OUT/progress.log"
  cp "$(find "$OUT/tl$i" -name '*kernel_stats.csv' | head -1)" "$OUT/tl${i}_kernel_stats.csv"
  rm -rf "$OUT/tl$i"
done
if [ -n "${LEG_AB:-}" ]; then
  for rep in $(seq 1 ${REPS:-1}); do
    for lib in ${LIBS:--}; do
      set -- $(run_leg "$LEG_AB")
      if [ "$lib" = "-" ]; then unset RLP_LIBRARY; else export RLP_LIBRARY=$ROOT/$lib; fi
      log "leg A/B rep $rep lib=$lib: $*"
      timeout -k 10 300 python -u scripts/leg.py "$@" > "$OUT/legab.log" 2>&1
      rc=$?; echo "{\"lib\": \"$lib\", \"rep\": $rep, \"out\": $(tail -1 "$OUT/legab.log")}" >> "$OUT/legab.jsonl"
      tail -1 "$OUT/legab.log" | cut -c1-300 | tee -a "$OUT/progress.log"
      step_rc $rc "leg A/B $lib"
    done
  done
  unset RLP_LIBRARY
fi
if [ "${FD_AB:-0}" = 1 ]; then
  i=0
  for rep in $(seq 1 ${REPS:-1}); do
    for lib in ${LIBS:--}; do
      i=$((i+1))
      if [ "$lib" = "-" ]; then unset RLP_LIBRARY; else export RLP_LIBRARY=$ROOT/$lib; fi
      log "FD A/B rep $rep lib=$lib"
      (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/fd$i" -o run \
          -- python3 "$ROOT/bench.py" --no-cpu-baseline --ddpg 0 --sac 0 --oa 0 --fp32-leg 0 --hbm 0 --uav 0 \
             --demo-e2e ${FD_DEMO:-0} --e2e 1 --e2e-k30 1 --steps 3 --warmup 1) > "$OUT/fd$i.log" 2>&1
      rc=$?; step_rc $rc "FD A/B $lib"
      kstats "$OUT/fd$i" | grep -E "ppo2_fd|ppo2_wgrad|rollout_sp|l1_|fg_grad|mfma_scale|mfma_pack|ppo2_reduce" > "$OUT/fd${i}_stats.txt"
      python3 - "$OUT/fd$i.log" "$lib" >> "$OUT/progress.log" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        d = json.loads(line)
        o = {"lib": sys.argv[2], "e2e_k6": d["e2e"]["s_per_iteration"], "e2e_k30": d["e2e"]["k30"]["s_per_iteration"]}
        for k in ("soi_ppo2_e2e", "ugvoa_ppo2_e2e"):
            if k in d: o[k] = d[k]["s_per_iteration"]
        print(json.dumps(o))
PY
      cat "$OUT/fd${i}_stats.txt" >> "$OUT/progress.log"; tail -8 "$OUT/progress.log"
      rm -rf "$OUT/fd$i"
    done
  done
  unset RLP_LIBRARY
fi
if [ -n "${BENCH:-}" ]; then
  log "bench $BENCH"
  timeout -k 10 600 python -u bench.py $BENCH > "$OUT/bench.log" 2>&1
  rc=$?; tail -1 "$OUT/bench.log" > "$OUT/bench.json"; tail -c 600 "$OUT/bench.log" | tee -a "$OUT/progress.log"
  step_rc $rc bench
fi
if [ -n "${BENCH_TRACE:-}" ]; then
  log "traced bench $BENCH_TRACE"
  (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/bt" -o run \
      -- python3 "$ROOT/bench.py" $BENCH_TRACE) > "$OUT/bench_traced.log" 2>&1
  rc=$?; tail -1 "$OUT/bench_traced.log" > "$OUT/bench_traced.json"; step_rc $rc "traced bench"
  kstats "$OUT/bt" > "$OUT/bt_stats.txt"; head -40 "$OUT/bt_stats.txt" | tee -a "$OUT/progress.log"
  cp "$(find "$OUT/bt" -name '*kernel_stats.csv' | head -1)" "$OUT/bt_kernel_stats.csv"
  if [ "${KEEP_TRACE:-0}" = 1 ]; then
    python3 scripts/trace_check.py "$OUT/bt" "$OUT/bench_traced.log" > "$OUT/trace_check.json" 2>&1 || true
  fi
  rm -rf "$OUT/bt"
fi
log DONE
