#!/bin/bash
# One gpurun call: GPU parity tests, a short bench, and a rocprofv3 kernel-trace profile.
# Every GPU step has its own time limit; a crash-type exit (abort/segv/timeout) ends the call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
TAG=${TAG:-r1}
mkdir -p "$OUT"
stop_on_crash() { rc=$1; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "STOP rc=$rc at $2"; exit "$rc"; fi; }

if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 ${PYTEST_ARGS:-} > "$OUT/gpu_tests_$TAG.log" 2>&1
  rc=$?; tail -25 "$OUT/gpu_tests_$TAG.log"; stop_on_crash $rc pytest
fi
if [ "${SKIP_BENCH:-0}" != 1 ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-600} python bench.py ${BENCH_ARGS:-} > "$OUT/bench_$TAG.log" 2>&1
  rc=$?; tail -3 "$OUT/bench_$TAG.log"; stop_on_crash $rc bench
fi
if [ "${SKIP_PROF:-0}" != 1 ]; then
  export TMPDIR=/tmp
  (cd /tmp && timeout -k 10 ${PROF_TIMEOUT:-600} rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$OUT/prof_$TAG" -o run -- python3 "$ROOT/bench.py" --steps 5 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-}) \
      > "$OUT/prof_$TAG.log" 2>&1
  rc=$?; tail -3 "$OUT/prof_$TAG.log"; stop_on_crash $rc rocprof
  find "$OUT/prof_$TAG" -name "*kernel_stats.csv" -exec head -20 {} \;
fi
echo DONE
