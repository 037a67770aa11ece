#!/bin/bash
# Where the 1-wave-per-SIMD rollout (physics mode 5, "cu4") wins: UAV at 32768 / 65536 envs and
# CartPole at 32768 envs against the auto choices; HIP-event launch times from the bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {  # tag, bench args...
  local tag=$1; shift
  timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --e2e 0 --ddpg 0 --oa 0 --sac 0 \
      --fp32-leg 0 "$@" > gpurun_out/sw_$tag.log 2>&1 || exit 1
  python3 - gpurun_out/sw_$tag.log "$tag" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
s = "%s cartpole %.3f ms %s" % (sys.argv[2], d["roofline"]["avg_launch_ms"], d["roofline"]["kernel"])
if "uav_ppo2_rollout" in d:
    u = d["uav_ppo2_rollout"]
    s += " | uav n=%d %.3f ms frac %.3f %s" % (u["envs_per_gpu"], u["roofline"]["avg_launch_ms"], u["roofline"]["frac"], u["roofline"]["kernel"])
print(s)
PY
}
run c64auto --uav 0
run c64cu64 --uav 0 --physics cu64
run c64auto2 --uav 0
run c64cu64b --uav 0 --physics cu64
run u64cu64 --uav 1 --uav-envs 65536 --uav-physics cu64
