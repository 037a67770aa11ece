#!/bin/bash
# rocprof A/B of the PPO2 FD kernel's block shape (RLP_FD_WAVES 4 vs 8) on the bench e2e leg.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
for W in ${VARIANTS:-W4 W8 W4}; do
  (cd /tmp && RLP_LIBRARY=$ROOT/reinforcementlearningplatform_amd/csrc/build/exp$W/librlp.so timeout -k 10 300 \
     rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_fd_$W" -o run -- python3 "$ROOT/bench.py" \
     --steps 2 --warmup 1 --no-cpu-baseline --e2e 2 --e2e-k30 0 --uav 0 --ddpg 0 --oa 0 --sac 0 --fp32-leg 0) \
     > "$OUT/b_fd_$W.log" 2>&1 || exit 1
  python3 - "$OUT/prof_fd_$W" "$W" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "ppo2_fd" in r["Name"] or "wgrad" in r["Name"]:
            print(sys.argv[2], r["Name"][:50], r["Calls"], "avg %.3f ms" % (float(r["AverageNs"]) / 1e6))
PY
done
