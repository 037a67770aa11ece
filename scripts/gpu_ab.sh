#!/bin/bash
# One gpurun call: rollout parity tests, then an A/B of bench.py variants (BENCH_A, BENCH_B args)
# under rocprofv3 kernel stats. Each GPU step has its own time limit; a crash stops the call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; TAG=${TAG:-ab}; mkdir -p "$OUT"
stop_on_crash() { rc=$1; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "STOP rc=$rc at $2"; exit "$rc"; fi; }
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/t_$TAG.log" 2>&1
  rc=$?; grep -E "FAILED|passed|failed" "$OUT/t_$TAG.log" | tail -15; stop_on_crash $rc pytest
fi
export TMPDIR=/tmp
i=0
for args in "${BENCH_A:-}" "${BENCH_B:-}" "${BENCH_C:-}" "${BENCH_D:-}"; do
  i=$((i+1)); [ -z "$args" ] && continue
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_${TAG}_$i" -o run \
      -- python3 "$ROOT/bench.py" --no-cpu-baseline --e2e 0 --ddpg 0 --oa 0 --sac 0 --fp32-leg 0 $args) > "$OUT/b_${TAG}_$i.log" 2>&1
  rc=$?; echo "== variant $i: $args (rc=$rc)"; tail -1 "$OUT/b_${TAG}_$i.log" | cut -c1-400; stop_on_crash $rc bench$i
  python3 - "$OUT/prof_${TAG}_$i" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "rollout" in r["Name"]:
            print("   ", r["Name"][:70], r["Calls"], "avg %.3f ms" % (float(r["AverageNs"]) / 1e6))
PY
done
echo DONE
