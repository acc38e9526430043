#!/bin/bash
# Round-4 GPU pass: every -m gpu test, smoke, the default bench line, then (optional)
# a 2-rank rehearsal of the N > 1 headline on the box's one GPU (BENCH_ONE_DEVICE).
# Each GPU step has its own time limit; a failing step ends the script (no retries).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r04}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rs --timeout 240 --timeout-method thread -p no:cacheprovider \
    ${PYTEST_ARGS:-} > gpurun_out/${TAG}_gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/${TAG}_gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as e; e.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/${TAG}_smoke.log
[ $rc -eq 0 ] || exit $rc
if [ -z "${NO_BENCH:-}" ]; then
  timeout -k 10 500 python -u bench.py --steps ${STEPS:-20} --warmup 5 ${BENCH_ARGS:-} > gpurun_out/${TAG}_bench.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -c 1500 gpurun_out/${TAG}_bench.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${REHEARSE:-}" ]; then
  BENCH_ONE_DEVICE=0 timeout -k 10 240 python -u bench.py --gpus 2 --steps 10 --warmup 2 --no-70b --no-collectives \
      --tg 0 > gpurun_out/${TAG}_rehearse.log 2>&1
  rc=$?; echo "rehearse rc=$rc"; tail -c 2500 gpurun_out/${TAG}_rehearse.log
fi
exit $rc
