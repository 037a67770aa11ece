#!/bin/bash
# Round 5: the r4i PMC command with the demo legs ON (the pass that crashed in round 4,
# profiles/r4/r4i_pmc_crash.txt), bench run under scripts/pmc_segv_diag.py so a SIGSEGV prints
# dladdr-named frames and /proc/self/maps. Each counter group its own rocprofv3 run; stop at the
# first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; TAG=${TAG:-r5a}; mkdir -p "$OUT/$TAG"
export TMPDIR=/tmp
ARGS=${PMC_BENCH_ARGS:-"--steps 2 --warmup 1 --no-cpu-baseline --ddpg 0 --oa 0 --sac 0 --fp32-leg 0 --e2e 1 --e2e-k30 0"}
DEFAULT_GROUPS='SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE GRBM_COUNT;SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VALU_TRANS_F32;FETCH_SIZE;WRITE_SIZE'
IFS=';' read -ra PGROUPS <<< "${PMC_GROUPS:-$DEFAULT_GROUPS}"
i=0
for group in "${PGROUPS[@]}"; do
  i=$((i+1))
  (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc $group --output-format csv -d "$OUT/$TAG/p$i" -o run \
      -- python3 "$ROOT/scripts/pmc_segv_diag.py" $ARGS) > "$OUT/$TAG/p$i.log" 2>&1
  rc=$?; echo "pass $i ($group) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/$TAG/p$i.log"; echo "STOP"; exit $rc; fi
done
python3 "$ROOT/scripts/parse_pmc.py" "$OUT/$TAG" > "$OUT/$TAG/pmc_summary.txt" 2>&1
grep -A22 -E "dense_gemm_kernel|chain3_|ppo2_dense_head|parts_reduce" "$OUT/$TAG/pmc_summary.txt" | head -150
echo DONE
