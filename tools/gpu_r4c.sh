set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_attn_oproj.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r04c_ao_tests.log 2>&1
rc=$?; echo "ao tests rc=$rc"; tail -15 gpurun_out/r04c_ao_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r04c_gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -5 gpurun_out/r04c_gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-large --no-70b --no-prefill > gpurun_out/r04c_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep -o '"value": [0-9.]*' gpurun_out/r04c_bench.log | head -1; grep -o '"llama3_8b": {[^}]*' gpurun_out/r04c_bench.log | head -c 400
exit $rc
