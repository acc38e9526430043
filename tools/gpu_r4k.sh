#!/bin/bash
# kq_mmq single-buffer occupancy experiment (lib/variants/libob4.so: KQ_MMQ_NBUF=1 + waves_per_eu 4;
# libob3.so: + waves_per_eu 3): prefill parity on the 64 x 64 tiles, then the prefill shapes on
# product AUTO / product tile64 / ob4 tile64 / ob3 tile64 / ob3 tile128, interleaved twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
V=$PWD/ggml-neon-opt_amd/lib/variants
MI355X_LIB=$V/libob4.so MI355X_MMQ_IMPL=tile64 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q \
    -k "mmq or prefill or batch" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r04k_tests.log 2>&1
rc=$?; echo "ob4 tests rc=$rc"; tail -2 gpurun_out/r04k_tests.log
[ $rc -eq 0 ] || exit $rc
: > gpurun_out/r04k_mmq.log
for r in 1 2; do
  for run in auto: tile64: tile64:ob4 tile64:ob3 tile128:ob3; do
    impl=${run%%:*}; name=${run#*:}; lib=""; [ -n "$name" ] && lib=$V/lib$name.so
    echo "== $impl ${name:-product} round $r" >> gpurun_out/r04k_mmq.log
    PREFILL_TYPES=12,13 MI355X_MMQ_IMPL=$impl MI355X_LIB=$lib timeout -k 10 150 python tools/prefill_bench.py \
        >> gpurun_out/r04k_mmq.log 2>&1 || exit $?
  done
done
grep -v amdgpu.ids gpurun_out/r04k_mmq.log | sed 's/total.*gemm/gemm/'
