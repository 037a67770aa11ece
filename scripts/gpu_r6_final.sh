#!/bin/bash
# Round 6 closing measurement: the whole GPU suite + smoke, the driver's bench command untraced
# and under the kernel trace (+ trace_check), the lidar leg traced, then FETCH_SIZE / WRITE_SIZE
# passes over an HBM-legs-only bench (profiles/pmc_traffic.json). Progress and a heartbeat go to
# gpurun_out/$TAG/progress.log; the first failing step ends the call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); TAG=${TAG:-r6fin}; OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"
export TAG
TESTS=all SMOKE=1 BENCH="--gpus 1 --steps 20 --warmup 5" BENCH_TRACE="--gpus 1 --steps 20 --warmup 5" \
    KEEP_TRACE=1 TRACE_LEGS="${TRACE_LEGS:-ugvoa_ppo2_leg}" bash scripts/gpu_r6.sh || exit $?
[ "${PMC:-1}" = 1 ] || exit 0
echo "[$(date +%T)] pmc passes" >> "$OUT/progress.log"
( while sleep 30; do echo "[$(date +%T)] alive" >> "$OUT/progress.log"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
i=0
for group in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $group --output-format csv -d "$OUT/pmc/p$i" -o run \
      -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --e2e 0 --uav 1 --fp32-leg 0 \
         --ddpg 0 --oa 0 --sac 0 --demo-e2e 0 --hbm 1) > "$OUT/pmc_p$i.log" 2>&1
  rc=$?; echo "[$(date +%T)] pmc pass $i ($group) rc=$rc" >> "$OUT/progress.log"
  [ $rc -ne 0 ] && exit $rc
done
python3 scripts/update_pmc_traffic.py "$OUT/pmc" "profiles/r6/${TAG}_pmc_summary.txt" \
    "$OUT/pmc_traffic.json" > "$OUT/pmc_summary.txt" 2>&1
echo "[$(date +%T)] pmc update rc=$?" >> "$OUT/progress.log"
python3 scripts/pmc_filter.py "$OUT/pmc" "rlp::" "$OUT/pmc_rlp_rows.csv" >> "$OUT/pmc_summary.txt" 2>&1
rm -rf "$OUT/pmc"
echo "[$(date +%T)] DONE" >> "$OUT/progress.log"
