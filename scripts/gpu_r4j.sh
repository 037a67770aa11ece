#!/bin/bash
# Round-4 calls j / k: where the DDPG tracking test parts (DIAG: libraries to compare), the full GPU
# suite on the variant V (not stopping at the first failure), then V's off-policy legs under a
# kernel trace + timelines, and the in-tree library's legs beside them.
#   j: DIAG="base exp4 exp6" V=exp6 (exp6 = exp4 + the fused data-only critic backward + the SAC
#      actor's trunk / heads chain); k: DIAG=exp7 V=exp7 (chains without per-tile branches)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; TAG=${TAG:-r4j}; mkdir -p "$OUT/$TAG"
export TMPDIR=/tmp
LIBD=reinforcementlearningplatform_amd/csrc/build
for v in ${DIAG:-base}; do
  if [ $v = base ]; then unset RLP_LIBRARY; else export RLP_LIBRARY=$ROOT/$LIBD/$v/librlp.so; fi
  timeout -k 10 180 python3 -u scripts/diag_ddpg_track.py 1000 > "$OUT/$TAG/diag_$v.log" 2>&1
  rc=$?; echo "diag $v rc=$rc"; tail -10 "$OUT/$TAG/diag_$v.log"; [ $rc -eq 0 ] || exit $rc
done
export RLP_LIBRARY=$ROOT/$LIBD/${V:-exp6}/librlp.so
timeout -k 10 700 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 200 \
   --timeout-method thread > "$OUT/$TAG/tests.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -12 "$OUT/$TAG/tests.log"
case $rc in 0|1) ;; *) exit $rc;; esac
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/$TAG/trace" -o run \
   -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --e2e 0 --e2e-k30 0 --demo-e2e 1 \
      --uav 0 --hbm 0 --fp32-leg 0 --oa 0 --ddpg 1 --sac 1) > "$OUT/$TAG/offpolicy_bench.log" 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/dispatch_timeline.py "$OUT/$TAG/trace" ddpg_td_kernel 20 6 30 > "$OUT/$TAG/ddpg_timeline.txt" 2>&1
python3 scripts/dispatch_timeline.py "$OUT/$TAG/trace" sac_target_kernel 20 12 48 > "$OUT/$TAG/sac_timeline.txt" 2>&1
tail -1 "$OUT/$TAG/ddpg_timeline.txt"; tail -1 "$OUT/$TAG/sac_timeline.txt"
rm -rf "$OUT/$TAG/trace"
unset RLP_LIBRARY
(cd /tmp && timeout -k 10 300 python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --e2e 0 --e2e-k30 0 \
   --demo-e2e 1 --uav 0 --hbm 0 --fp32-leg 0 --oa 0 --ddpg 1 --sac 1) > "$OUT/$TAG/offpolicy_bench_base.log" 2>&1
rc=$?; echo "base bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 - "$OUT/$TAG/offpolicy_bench.log" "$OUT/$TAG/offpolicy_bench_base.log" <<'PY'
import json, sys
for f in sys.argv[1:]:
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l)
            print(f.split("/")[-1], {k: {x: d[k].get(x) for x in ("value", "learn_ms", "s_per_iteration")}
                                     for k in ("soi_ddpg", "ugvoa_sac", "soi_ppo2_e2e", "ugvoa_ppo2_e2e") if k in d})
PY
echo DONE
