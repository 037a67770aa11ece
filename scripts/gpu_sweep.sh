#!/bin/bash
# Run the GPU tests (unless SKIP_TESTS=1) then bench.py once per item of SWEEP (';'-separated
# bench.py argument strings), printing value / rollout time / MFMA fraction.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out; mkdir -p "$OUT"; TAG=${TAG:-sweep}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 ${PYTEST_ARGS:-} > "$OUT/gpu_tests_$TAG.log" 2>&1
  rc=$?; tail -3 "$OUT/gpu_tests_$TAG.log"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
IFS=';' read -ra ITEMS <<< "${SWEEP:---precision f16x3}"
i=0
for item in "${ITEMS[@]}"; do
  i=$((i+1))
  timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} $item > "$OUT/bench_${TAG}_$i.log" 2>&1 || { echo "STOP at $item"; exit 1; }
  tail -1 "$OUT/bench_${TAG}_$i.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$item', 'value %.4e'%d['value'], 'rollout_ms %.2f'%d['roofline']['avg_launch_ms'], 'frac %.3f'%d['roofline']['frac'], 'ms/step %.2f'%d['ms_per_step'])"
done
echo DONE
