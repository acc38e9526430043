#!/bin/bash
# kq_mmf (f16 prefill path): GPU tests, then the prefill shapes on both precisions.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_mmf.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/mmf_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 gpurun_out/mmf_tests.log
[ $rc -eq 0 ] || exit $rc
MI355X_PREFILL=f16 timeout -k 10 200 python -u tools/prefill_bench.py > gpurun_out/mmf_bench_f16.log 2>&1
rc=$?; echo "bench f16 rc=$rc"; cat gpurun_out/mmf_bench_f16.log | grep -v amdgpu.ids
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/prefill_bench.py > gpurun_out/mmf_bench_exact.log 2>&1
rc=$?; echo "bench exact rc=$rc"; cat gpurun_out/mmf_bench_exact.log | grep -v amdgpu.ids
exit $rc
