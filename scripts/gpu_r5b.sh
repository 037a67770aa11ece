#!/bin/bash
# Round 5: counters and per-shape durations for the dense-GEMM / chain kernels (the demo-net PPO2
# updates and the off-policy learn()s). One kernel-trace pass and one rocprofv3 --pmc pass per
# counter group over the same short bench, each its own run with its own time limit; after each
# pass only the rows of the kernels of interest are kept (gpurun_out <= 64 MiB). A heartbeat line
# every 60 s keeps the run visibly alive (a --pmc pass prints nothing until the bench ends).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; TAG=${TAG:-r5b}; mkdir -p "$OUT/$TAG"
export TMPDIR=/tmp
ARGS=${PMC_BENCH_ARGS:-"--steps 2 --warmup 1 --no-cpu-baseline --fp32-leg 0 --e2e 1 --e2e-k30 0 --uav 0 --hbm 0 --offpolicy-steps 3"}
PAT=${PAT:-"dense_gemm|chain3|ppo2_dense_head|parts_reduce|adam_reduce|wgrad_reduce|ppo2_fd|ppo2_wgrad|rollout_sp|packed_forward|mlp_forward"}
( while sleep 60; do echo "alive $(date +%T)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
if [ "${SKIP_TRACE:-0}" != 1 ]; then
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$TAG/trace" -o run \
      -- python3 "$ROOT/scripts/pmc_segv_diag.py" $ARGS) > "$OUT/$TAG/trace.log" 2>&1
  rc=$?; echo "trace rc=$rc"; tail -c 300 "$OUT/$TAG/trace.log"; echo
  [ $rc -ne 0 ] && exit $rc
  python3 "$ROOT/scripts/trace_shapes.py" "$OUT/$TAG/trace" "$PAT" > "$OUT/$TAG/trace_shapes.txt"
  cp "$(find "$OUT/$TAG/trace" -name '*kernel_stats.csv' | head -1)" "$OUT/$TAG/kernel_stats.csv"
  rm -rf "$OUT/$TAG/trace"
fi
DEFAULT_GROUPS='SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE GRBM_COUNT;SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VALU_TRANS_F32;FETCH_SIZE;WRITE_SIZE'
IFS=';' read -ra PGROUPS <<< "${PMC_GROUPS:-$DEFAULT_GROUPS}"
i=0
rc=0
for group in "${PGROUPS[@]}"; do
  i=$((i+1))
  (cd /tmp && timeout -s KILL 400 rocprofv3 --pmc $group --output-format csv -d "$OUT/$TAG/p$i" -o run \
      -- python3 "$ROOT/scripts/pmc_segv_diag.py" $ARGS) > "$OUT/$TAG/p$i.log" 2>&1
  rc=$?; echo "pass $i ($group) rc=$rc $(date +%T)"
  python3 "$ROOT/scripts/pmc_filter.py" "$OUT/$TAG/p$i" "$PAT" "$OUT/$TAG/p${i}_filtered.csv"
  rm -rf "$OUT/$TAG/p$i"
  if [ $rc -ne 0 ]; then tail -c 20000 "$OUT/$TAG/p$i.log" > "$OUT/$TAG/p${i}_tail.log"; tail -5 "$OUT/$TAG/p$i.log"; echo "STOP"; break; fi
  tail -c 2000 "$OUT/$TAG/p$i.log" > "$OUT/$TAG/p${i}_tail.log"; rm -f "$OUT/$TAG/p$i.log"
done
python3 "$ROOT/scripts/parse_pmc.py" "$OUT/$TAG" --by-grid "$PAT" > "$OUT/$TAG/pmc_summary.txt" 2>&1
[ $rc -ne 0 ] && exit $rc
sed -n '/# per launch shape/,$p' "$OUT/$TAG/pmc_summary.txt" | head -60
head -30 "$OUT/$TAG/trace_shapes.txt"
echo DONE
