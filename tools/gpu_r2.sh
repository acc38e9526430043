set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_mmf.py tests/test_gpu_ops.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/t2.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/t2.log
[ $rc -eq 0 ] || exit $rc
for cfg in "MI355X_GEMV_PRE0=1" "MI355X_LIB=ggml-neon-opt_amd/lib/variants/libdq4.so" "MI355X_GEMV_PRE0=3" "MI355X_GEMV_WPC=8" "MI355X_LIB=ggml-neon-opt_amd/lib/variants/libdq4.so MI355X_GEMV_WPC=8" "MI355X_GEMV_PRE0=1" "MI355X_LIB=ggml-neon-opt_amd/lib/variants/libdq4.so" "MI355X_GEMV_WPC=8"; do echo "== $cfg"; env $cfg timeout -k 10 120 python -u tools/gemv_large_ab.py 2>&1 | grep -v amdgpu.ids || exit 1; done
