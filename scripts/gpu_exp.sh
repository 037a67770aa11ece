#!/bin/bash
# Timing experiments: bench.py's rollout launch time with librlp variants built with
# -DRLP_EXPERIMENT=<k> (csrc/build/exp<k>/librlp.so; parts of the kernel removed, results invalid).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
L=reinforcementlearningplatform_amd/librlp.so; cp $L /tmp/librlp_main.so
for X in main ${EXPS:-1 2}; do
  if [ $X = main ]; then cp /tmp/librlp_main.so $L; else cp reinforcementlearningplatform_amd/csrc/build/exp$X/librlp.so $L; fi
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --e2e 0 --uav 0 --fp32-leg 0 ${BENCH_ARGS:-} > gpurun_out/exp_$X.log 2>&1 || { echo "STOP $X"; exit 1; }
  tail -1 gpurun_out/exp_$X.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$X', 'rollout_ms %.3f'%d['roofline']['avg_launch_ms'])"
done
cp /tmp/librlp_main.so $L
