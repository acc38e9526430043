#!/bin/bash
# Prefill GEMM ablations (timing only) of kq_mmq<Q4_K>: KQ_MMQ_DIAG values in $DIAGS, kernel
# variant $IMPL. The diagnostics are compile time; build each library on the CPU first:
#   make -C ggml-neon-opt_amd variant-mmq NAME=mmqd13 VFLAGS=-DKQ_MMQ_DIAG=13
# (diag 0 = the product library).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; : > gpurun_out/mmqdiag.log
for d in ${DIAGS:-0 13 16}; do
    lib=""; [ "$d" != 0 ] && lib="ggml-neon-opt_amd/lib/variants/libmmqd$d.so"
    echo "diag $d" >> gpurun_out/mmqdiag.log
    PREFILL_TYPES=${PREFILL_TYPES:-12} MI355X_MMQ_IMPL=${IMPL:-auto} MI355X_LIB=$lib \
        timeout -k 10 120 python tools/prefill_bench.py >> gpurun_out/mmqdiag.log 2>&1 || exit $?
done
cat gpurun_out/mmqdiag.log
