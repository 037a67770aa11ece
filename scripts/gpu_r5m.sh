#!/bin/bash
# Round 5 closing measurement, part 1: GPU suite + smoke, the driver's bench command untraced, then
# the same command under rocprofv3 --kernel-trace --stats with scripts/trace_check.py over it (the
# trace CSV is reduced to the bench's hot-path kernels before the copy back).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); T=${TAG:-r5m}; OUT=$ROOT/gpurun_out/$T; mkdir -p "$OUT"
export TMPDIR=/tmp
TAG=$T bash scripts/gpu_tests.sh || exit $?
TAG=$T bash scripts/gpu_bench.sh || exit $?
( while sleep 60; do echo "alive $(date +%T)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run \
    -- python3 "$ROOT/bench.py" --gpus 1 --steps 20 --warmup 5) > "$OUT/trace_bench.log" 2>&1
rc=$?; tail -c 400 "$OUT/trace_bench.log"; echo; echo "trace rc=$rc"
[ $rc -ne 0 ] && exit $rc
python3 "$ROOT/scripts/trace_check.py" "$OUT/trace" "$OUT/trace_bench.log" > "$OUT/trace_check.json"
head -30 "$OUT/trace_check.json"
cp "$(find "$OUT/trace" -name '*kernel_stats.csv' | head -1)" "$OUT/kernel_stats.csv"
python3 "$ROOT/scripts/trace_shapes.py" "$OUT/trace" "rollout_sp|ppo2_fd|ppo2_wgrad|fg_grad|l1_fwd|l1_wgrad|ppo2_reduce|dense_gemm|chain3|gae|reward" > "$OUT/trace_shapes.txt"
rm -rf "$OUT/trace"
echo DONE
