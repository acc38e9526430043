#!/bin/bash
# One GPU-box pass: every -m gpu test, smoke, then the bench (default line and
# optional extra bench args). Each GPU step has its own time limit; a failing step
# ends the script (no retries). Logs under gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider \
    ${PYTEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as e; e.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps ${STEPS:-20} --warmup 5 ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 4000 gpurun_out/bench.log
[ $rc -eq 0 ] || exit $rc
if [ -n "${BENCH2_ARGS:-}" ]; then
  timeout -k 10 300 python -u bench.py --steps ${STEPS:-20} --warmup 5 $BENCH2_ARGS > gpurun_out/bench2.log 2>&1
  rc=$?; echo "bench2 rc=$rc"; tail -c 3000 gpurun_out/bench2.log
fi
exit $rc
