#!/bin/bash
# Timing A/B builds (load one with RLP_LIBRARY=<path> python bench.py ...): librlp.so from the csrc sources in SRC_DIR (default:
# this tree's) with extra hipcc flags, into csrc/build/exp<X>/librlp.so.
#   scripts/build_variant.sh X [SRC_DIR] [hipcc flags...]
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
X=$1; shift
SRC=$R/reinforcementlearningplatform_amd/csrc
if [ $# -gt 0 ] && [ -d "$1" ]; then SRC=$1; shift; fi
OUT=$R/reinforcementlearningplatform_amd/csrc/build/exp$X
mkdir -p "$OUT"
printf '%s\n' rlp_env rlp_mlp rlp_rollout rlp_learn rlp_update rlp_replay rlp_lidar |
  xargs -P 7 -I{} /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -ffp-contract=off \
      -munsafe-fp-atomics -w "$@" -c "$SRC/{}.hip" -o "$OUT/{}.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT/librlp.so" "$OUT"/rlp_*.o \
    -Wl,-rpath,/opt/rocm/lib
echo "$OUT/librlp.so"
