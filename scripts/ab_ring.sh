#!/bin/bash
# rocprof A/B of rollout build variants (csrc/build/exp<V>/librlp.so, scripts/build_variant.sh) on the bench rollout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
for V in ${VARIANTS:-R3 R4 R3 R4}; do
  (cd /tmp && RLP_LIBRARY=$ROOT/reinforcementlearningplatform_amd/csrc/build/exp$V/librlp.so timeout -k 10 300 \
     rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_ab_$V" -o run -- python3 "$ROOT/bench.py" \
     --steps 5 --warmup 2 --no-cpu-baseline --e2e 0 --uav ${UAV:-0} --ddpg 0 --oa 0 --sac 0 --fp32-leg 0) \
     > "$OUT/b_ab_$V.log" 2>&1 || exit 1
  python3 - "$OUT/prof_ab_$V" "$V" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "rollout" in r["Name"]:
            print(sys.argv[2], r["Name"][:50], r["Calls"], "avg %.3f ms" % (float(r["AverageNs"]) / 1e6))
PY
done
