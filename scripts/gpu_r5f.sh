#!/bin/bash
# Round 5: the 41-input nets' f16x3 update (EXT kernels) + the dense GEMM's LDS layout: the update
# tests first (a fault stops here), then the whole GPU suite + smoke, then trace + counters.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r5f}; mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_plain_nets.py -x -v --timeout 120 --timeout-method thread > "$OUT/plain_nets.log" 2>&1
rc=$?; grep -E "PASS|FAIL|Error|error|native err" "$OUT/plain_nets.log" | tail -30; echo "plain_nets rc=$rc"
[ $rc -ne 0 ] && exit $rc
TAG=${TAG:-r5f} bash scripts/gpu_tests.sh || exit $?
TAG=${TAG:-r5f} bash scripts/gpu_r5b.sh
