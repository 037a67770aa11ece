#!/bin/bash
# Round-4 measurement, part 2: the issue / LDS / HBM counter passes (one rocprofv3 --pmc run per
# group, no trace domains) over a short bench, summarised by scripts/parse_pmc.py. The demo-net
# legs stay off: a dense-GEMM launch under --pmc crashed inside the profiler-wrapped runtime
# (profiles/r4/r4i_pmc_crash.txt); those legs have no counters to collect here.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r4i} SKIP_TRACE=1 PMC_BENCH_ARGS="--steps 2 --warmup 1 --no-cpu-baseline --ddpg 0 --oa 0 --sac 0 --fp32-leg 0 --e2e 1 --e2e-k30 0 --demo-e2e 0" bash scripts/gpu_measure.sh
