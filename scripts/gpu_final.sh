set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/r3w
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests > gpurun_out/r3w/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r3w/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r3w/smoke.log 2>&1
rc=$?; tail -2 gpurun_out/r3w/smoke.log; [ $rc -ne 0 ] && exit $rc
TAG=r3w bash scripts/gpu_measure.sh
