#!/bin/bash
# One gpurun call: same-box A/B of librlp builds (LIBS: space-separated paths, "-" = the in-tree
# library) on one bench.py command (ARGS) under rocprofv3 kernel stats; prints the average
# duration of every kernel whose name matches PAT. Each GPU step has its own time limit; a crash
# stops the script.  e.g. LIBS="- csrc/build/exp1/librlp.so" ARGS="--e2e 1" PAT="fd|wgrad"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); TAG=${TAG:-lab}; OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
BASE="--no-cpu-baseline --ddpg 0 --sac 0 --oa ${OA:-0} --fp32-leg 0 --hbm 0 --uav 0 --e2e 0 --e2e-k30 0 --demo-e2e 0"
i=0
for rep in $(seq 1 ${REPS:-1}); do
for lib in ${LIBS:--}; do
  i=$((i+1))
  if [ "$lib" = "-" ]; then unset RLP_LIBRARY; else export RLP_LIBRARY=$ROOT/$lib; fi
  (cd /tmp && timeout -k 10 ${BT:-300} rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/p$i" -o run \
      -- python3 "$ROOT/bench.py" $BASE ${ARGS:-}) > "$OUT/b$i.log" 2>&1
  rc=$?; echo "== $i lib=$lib rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/b$i.log"; exit $rc; fi
  python3 - "$OUT/p$i" "$OUT/b$i.log" "${PAT:-.}" <<'PY'
import csv, glob, json, re, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if re.search(sys.argv[3], r["Name"]):
            print("   %-70s %5s avg %.4f ms" % (r["Name"][:70], r["Calls"], float(r["AverageNs"]) / 1e6))
for line in open(sys.argv[2]):
    if line.startswith("{"):
        d = json.loads(line)
        o = {"rollout_ms": round(d["roofline"]["avg_launch_ms"], 4)}
        if "e2e" in d:
            o["e2e"] = round(d["e2e"]["s_per_iteration"], 4)
            if "k30" in d["e2e"]: o["e2e_k30"] = round(d["e2e"]["k30"]["s_per_iteration"], 4)
        for k in ("soi_ppo2_e2e", "ugvoa_ppo2_e2e"):
            if k in d and "s_per_iteration" in d[k]: o[k] = round(d[k]["s_per_iteration"], 4)
        if "ugvoa_ppo2_rollout" in d: o["ugvoa_rollout"] = "%.4g" % d["ugvoa_ppo2_rollout"]["value"]
        if "uav_ppo2_rollout" in d: o["uav_ms"] = round(d["uav_ppo2_rollout"]["roofline"]["avg_launch_ms"], 4)
        print("   ", json.dumps(o))
PY
done
done
echo DONE
