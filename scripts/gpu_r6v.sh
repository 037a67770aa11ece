#!/bin/bash
# Round 6 (v): where l1_fwd_kernel's time goes: the UGV-OA PPO2 demo iteration under the kernel
# trace on the in-tree build and on three timing-only diagnostic builds (RLP_L1_DIAG: 1 no tanh,
# 2 no h1 stores, 3 no layer-1 MFMAs; wrong results by construction, never shipped).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); TAG=${TAG:-r6v}; OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
( while sleep 30; do echo "[$(date +%T)] alive" >> "$OUT/progress.log"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
for v in - l1d1 l1d2 l1d3; do
  if [ "$v" = - ]; then unset RLP_LIBRARY; else export RLP_LIBRARY=$ROOT/reinforcementlearningplatform_amd/csrc/build/exp$v/librlp.so; fi
  echo "[$(date +%T)] trace $v" >> "$OUT/progress.log"
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/t_$v" -o run \
      -- python3 "$ROOT/scripts/leg.py" demo_nets_e2e_leg which=ugvoa) > "$OUT/t_$v.log" 2>&1
  rc=$?; unset RLP_LIBRARY
  [ $rc -ne 0 ] && { echo "STOP $v rc=$rc" >> "$OUT/progress.log"; exit $rc; }
  python3 - "$OUT/t_$v" "$v" <<'PY' >> "$OUT/progress.log"
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if any(k in r["Name"] for k in ("l1_fwd", "l1_wgrad", "ppo2_fd_kernel<0", "ppo2_wgrad_kernel<0")):
        print(sys.argv[2], r["Name"][:40], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1))
PY
  rm -rf "$OUT/t_$v"
done
echo "[$(date +%T)] DONE" >> "$OUT/progress.log"
