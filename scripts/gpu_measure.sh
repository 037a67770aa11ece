#!/bin/bash
# One gpurun call: rocprofv3 kernel trace of EXACTLY the driver's bench command
# (`bench.py --gpus 1 --steps 20 --warmup 5`), the trace-vs-bench check (scripts/trace_check.py),
# then issue / LDS / HBM counter passes over a short bench (one rocprofv3 --pmc run per group,
# no trace domains combined with --pmc). Every GPU step has its own time limit and the script
# stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; TAG=${TAG:-r3a}; mkdir -p "$OUT/$TAG"
export TMPDIR=/tmp
BENCH=${BENCH_CMD:-"--gpus 1 --steps 20 --warmup 5"}
if [ "${SKIP_TRACE:-0}" != 1 ]; then
  (cd /tmp && timeout -k 10 480 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$TAG/trace" -o run \
      -- python3 "$ROOT/bench.py" $BENCH) > "$OUT/$TAG/trace_bench.log" 2>&1
  rc=$?; tail -c 600 "$OUT/$TAG/trace_bench.log"; echo; echo "trace rc=$rc"
  [ $rc -ne 0 ] && exit $rc
  python3 "$ROOT/scripts/trace_check.py" "$OUT/$TAG/trace" "$OUT/$TAG/trace_bench.log" > "$OUT/$TAG/trace_check.json"
  head -40 "$OUT/$TAG/trace_check.json"
fi
ARGS=${PMC_BENCH_ARGS:-"--steps 2 --warmup 1 --no-cpu-baseline --ddpg 0 --oa 0 --sac 0 --fp32-leg 0 --e2e 1 --e2e-k30 0"}
DEFAULT_GROUPS='SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE GRBM_COUNT;SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VALU_TRANS_F32;FETCH_SIZE;WRITE_SIZE'
IFS=';' read -ra PGROUPS <<< "${PMC_GROUPS:-$DEFAULT_GROUPS}"
i=0
for group in "${PGROUPS[@]}"; do
  i=$((i+1))
  [ "${SKIP_PMC:-0}" = 1 ] && break
  (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $group --output-format csv -d "$OUT/$TAG/p$i" -o run \
      -- python3 "$ROOT/bench.py" $ARGS) > "$OUT/$TAG/p$i.log" 2>&1
  rc=$?; echo "pass $i ($group) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/$TAG/p$i.log"; echo "STOP"; exit $rc; fi
done
if [ "${SKIP_PMC:-0}" != 1 ]; then
  python3 "$ROOT/scripts/parse_pmc.py" "$OUT/$TAG" > "$OUT/$TAG/pmc_summary.txt" 2>&1
  grep -A30 -E "rollout_sp_kernel|ppo2_fd_kernel" "$OUT/$TAG/pmc_summary.txt" | head -120
fi
echo DONE
