#!/bin/bash
# PMC passes over a short bench run (each counter group in its own rocprofv3 run; no trace
# domains combined with --pmc).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; TAG=${TAG:-pmc}; mkdir -p "$OUT/$TAG"
export TMPDIR=/tmp
ARGS=${BENCH_ARGS:-"--steps 2 --warmup 1 --no-cpu-baseline"}
(cd /tmp && timeout -k 10 120 rocprofv3 -L > "$OUT/$TAG/counters_list.txt" 2>&1) || true
i=0
DEFAULT_GROUPS='FETCH_SIZE;WRITE_SIZE;SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES;SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY;SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM;TCC_HIT_sum TCC_MISS_sum'
IFS=';' read -ra PGROUPS <<< "${PMC_GROUPS:-$DEFAULT_GROUPS}"
for group in "${PGROUPS[@]}"; do
  i=$((i+1))
  (cd /tmp && timeout -k 10 300 rocprofv3 --pmc $group --output-format csv -d "$OUT/$TAG/p$i" -o run \
      -- python3 "$ROOT/bench.py" $ARGS) > "$OUT/$TAG/p$i.log" 2>&1
  rc=$?; echo "pass $i ($group) rc=$rc"; tail -2 "$OUT/$TAG/p$i.log"
  if [ $rc -ne 0 ]; then echo "STOP"; exit $rc; fi
done
python3 "$ROOT/scripts/parse_pmc.py" "$OUT/$TAG" > "$OUT/$TAG/summary.txt" 2>&1; cat "$OUT/$TAG/summary.txt"
echo DONE
