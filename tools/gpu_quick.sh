set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_mmf.py tests/test_gpu_ops.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/t1.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/t1.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-large --no-70b > gpurun_out/b1.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 300 gpurun_out/b1.log
exit $rc
