#!/bin/bash
# UAV rollout leg under two rollout kernels (bench --uav-physics), alternated; HIP-event launch times.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for M in ${MODES:-auto cu4 auto cu4}; do
  timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --e2e 0 --ddpg 0 --oa 0 --sac 0 \
      --fp32-leg 0 --uav 1 --uav-physics "$M" > gpurun_out/b_uav_$M.log 2>&1 || exit 1
  python3 - gpurun_out/b_uav_$M.log "$M" <<'PY'
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith("{")][-1]
d = json.loads(line)
u = d["uav_ppo2_rollout"]
print(sys.argv[2], "cartpole %.3f ms" % d["roofline"]["avg_launch_ms"], "uav %.3f ms" % u["roofline"]["avg_launch_ms"],
      "frac %.3f" % u["roofline"]["frac"], u["roofline"]["kernel"])
PY
done
