#!/bin/bash
# Timing A/B builds (load one with RLP_LIBRARY=<path> python bench.py ...): librlp.so with the
# listed csrc sources recompiled with extra hipcc flags (the other objects from the main build,
# csrc/build/*.o — run make first), into csrc/build/exp<X>/librlp.so.
#   scripts/build_variant.sh X "rlp_update rlp_rollout" [hipcc flags...]
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
X=$1; FILES=$2; shift 2
SRC=$R/reinforcementlearningplatform_amd/csrc
OUT=$SRC/build/exp$X
mkdir -p "$OUT"
cp "$SRC"/build/rlp_*.o "$OUT"/
for f in $FILES; do
  extra=""
  [ "$f" = rlp_update ] && [ -z "${SLP:-}" ] && extra=-fno-slp-vectorize
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -ffp-contract=off \
      -munsafe-fp-atomics -w $extra "$@" -c "$SRC/$f.hip" -o "$OUT/$f.o" &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT/librlp.so" "$OUT"/rlp_*.o \
    -Wl,-rpath,/opt/rocm/lib
echo "$OUT/librlp.so"
