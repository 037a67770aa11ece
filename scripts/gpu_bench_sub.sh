#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out; mkdir -p "$OUT"; TAG=${TAG:-x}
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 > "$OUT/gpu_tests_$TAG.log" 2>&1
rc=$?; tail -5 "$OUT/gpu_tests_$TAG.log"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for sub in 4 2; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --sub $sub --no-cpu-baseline > "$OUT/bench_${TAG}_sub$sub.log" 2>&1 || exit $?
  tail -1 "$OUT/bench_${TAG}_sub$sub.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('sub', $sub, 'value %.3e'%d['value'], 'rollout_ms %.2f'%d['roofline']['avg_launch_ms'], 'frac %.3f'%d['roofline']['frac'], 'ms/step %.2f'%d['ms_per_step'])"
done
echo DONE
