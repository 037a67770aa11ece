#!/bin/bash
# Kernel-trace stats of a short e2e bench (rollout + GAE + native PPO2 update), then optional PMC
# passes (PMC_GROUPS, ';'-separated) over the same command.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; TAG=${TAG:-e2e}; mkdir -p "$OUT/$TAG"
export TMPDIR=/tmp
ARGS=${BENCH_ARGS:-"--steps 2 --warmup 1 --no-cpu-baseline --uav 0 --ddpg 0 --oa 0 --sac 0 --fp32-leg 0 --e2e 1"}
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$TAG/ks" -o run \
    -- python3 "$ROOT/bench.py" $ARGS) > "$OUT/$TAG/ks.log" 2>&1
rc=$?; echo "kernel stats rc=$rc"; [ $rc -ne 0 ] && exit $rc
find "$OUT/$TAG/ks" -name "*kernel_stats.csv" -exec head -12 {} \; | cut -c1-160
if [ -n "${PMC_GROUPS:-}" ]; then
  IFS=';' read -ra PG <<< "$PMC_GROUPS"; i=0
  for group in "${PG[@]}"; do
    i=$((i+1))
    (cd /tmp && timeout -k 10 300 rocprofv3 --pmc $group --output-format csv -d "$OUT/$TAG/p$i" -o run \
        -- python3 "$ROOT/bench.py" $ARGS) > "$OUT/$TAG/p$i.log" 2>&1
    rc=$?; echo "pass $i rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
  python3 "$ROOT/scripts/parse_pmc.py" "$OUT/$TAG" > "$OUT/$TAG/summary.txt" 2>&1
  grep -A20 "ppo2_fd_kernel<1, 1, 0>" "$OUT/$TAG/summary.txt"
fi
echo DONE
