#!/bin/bash
# kq_mmq with the Q4_K fp32 chain on packed f32 (lib/variants/libpk.so, KQ_MMQ_PKCHAIN=1): prefill
# parity on every tile, then the Q4_K prefill shapes, product vs pk, interleaved twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
V=$PWD/ggml-neon-opt_amd/lib/variants
for L in pk pk7; do
MI355X_LIB=$V/lib$L.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ops.py -x -q \
    -k "mmq or prefill or batch or prompt" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r04o_tests.log 2>&1
rc=$?; echo "$L tests rc=$rc"; tail -2 gpurun_out/r04o_tests.log
[ $rc -eq 0 ] || exit $rc
done
: > gpurun_out/r04o_mmq.log
for r in 1 2; do
  for name in "" pk pk7; do
    lib=""; [ -n "$name" ] && lib=$V/lib$name.so
    echo "== ${name:-product} round $r" >> gpurun_out/r04o_mmq.log
    MI355X_LIB=$lib timeout -k 10 150 python tools/prefill_bench.py >> gpurun_out/r04o_mmq.log 2>&1 || exit $?
  done
done
grep -v amdgpu.ids gpurun_out/r04o_mmq.log | sed 's/total.*gemm/gemm/'
