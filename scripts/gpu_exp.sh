#!/bin/bash
# Timing experiments: bench.py with librlp variants built with -DRLP_EXPERIMENT=<k>
# (csrc/build/exp<k>/librlp.so: parts of a kernel removed, results invalid), profiled with
# rocprofv3 --kernel-trace --stats; prints the top kernels of each variant.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out
L=reinforcementlearningplatform_amd/librlp.so; cp $L /tmp/librlp_main.so
export TMPDIR=/tmp
for X in main ${EXPS:-1}; do
  if [ $X = main ]; then cp /tmp/librlp_main.so $L; else cp reinforcementlearningplatform_amd/csrc/build/exp$X/librlp.so $L; fi
  rm -rf gpurun_out/exp_$X; mkdir -p gpurun_out/exp_$X
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/exp_$X -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --uav 0 --fp32-leg 0 ${BENCH_ARGS:-}) > gpurun_out/exp_$X.log 2>&1 || { echo "STOP $X"; cp /tmp/librlp_main.so $L; exit 1; }
  f=$(find gpurun_out/exp_$X -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:${TOPK:-4}]:
    print('$X', r['Name'][:60], 'avg_ms=%.3f'%(float(r['AverageNs'])/1e6))
"
done
cp /tmp/librlp_main.so $L
