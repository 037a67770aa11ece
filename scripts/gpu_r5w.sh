#!/bin/bash
# Round 5: timing-only diagnostics of ppo2_wgrad_kernel (wrong gradients by construction, never
# shipped): no h1 fragment build after the first tile (expNB), no G2 loads after the first tile
# (expNL), neither (expNBL), against the in-tree kernel.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${TAG:-r5w}; C=reinforcementlearningplatform_amd/csrc/build
TAG=$T/ab REPS=${REPS:-2} LIBS="- $C/expNB/librlp.so $C/expNL/librlp.so $C/expNBL/librlp.so" \
  ARGS="--e2e 1 --e2e-k30 0 --demo-e2e 0" PAT="wgrad_kernel<1" bash scripts/gpu_lib_ab.sh
