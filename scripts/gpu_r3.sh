#!/bin/bash
# Round-3 GPU check: selected GPU tests, then short benches (each step time-limited, stop on crash).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r3}; mkdir -p "$OUT"
stop() { rc=$1; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "STOP rc=$rc at $2"; exit "$rc"; fi; }
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread \
      -p no:cacheprovider $TESTS > "$OUT/tests.log" 2>&1
  rc=$?; tail -12 "$OUT/tests.log"; stop $rc pytest
fi
i=0
IFS=';' read -ra BENCHES <<< "${BENCH_SETS:-}"
for b in "${BENCHES[@]}"; do
  i=$((i+1))
  timeout -k 10 ${BENCH_TIMEOUT:-400} python bench.py $b > "$OUT/bench$i.log" 2>&1
  rc=$?; echo "bench $i ($b) rc=$rc"; tail -c 2500 "$OUT/bench$i.log"; echo; stop $rc bench$i
done
echo DONE
