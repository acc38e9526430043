#!/bin/bash
# Prefill GEMM A/B over libraries and kernel selectors: RUNS="impl:lib ..." (lib "" = the
# product library, else ggml-neon-opt_amd/lib/variants/lib<name>.so), shapes of
# tools/prefill_bench.py filtered by PREFILL_TYPES.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; : > gpurun_out/mmq_libs.log
for run in ${RUNS:-tile64: k4:}; do
    impl=${run%%:*}; name=${run#*:}; lib=""; [ -n "$name" ] && lib="ggml-neon-opt_amd/lib/variants/lib$name.so"
    echo "== impl $impl lib ${name:-product}" >> gpurun_out/mmq_libs.log
    PREFILL_TYPES=${PREFILL_TYPES:-12} MI355X_MMQ_IMPL=$impl MI355X_LIB=$lib \
        timeout -k 10 120 python tools/prefill_bench.py >> gpurun_out/mmq_libs.log 2>&1 || exit $?
done
grep -v amdgpu.ids gpurun_out/mmq_libs.log | sed 's/total.*gemm/gemm/'
