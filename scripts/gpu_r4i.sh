#!/bin/bash
# Round-4 measurement, part 2: the issue / LDS / HBM counter passes (one rocprofv3 --pmc run per
# group, no trace domains) over a short bench, summarised by scripts/parse_pmc.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r4i} SKIP_TRACE=1 bash scripts/gpu_measure.sh
