#!/bin/bash
# Prefill GEMM ablations (timing only): MI355X_MMQ_DIAG values in $DIAGS, variant $IMPL.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; : > gpurun_out/mmqdiag.log
for d in ${DIAGS:-0 13 16}; do echo "diag $d" >> gpurun_out/mmqdiag.log; PREFILL_TYPES=${PREFILL_TYPES:-12} MI355X_MMQ_IMPL=${IMPL:-auto} MI355X_MMQ_DIAG=$d timeout -k 10 120 python tools/prefill_bench.py >> gpurun_out/mmqdiag.log 2>&1 || exit $?; done
cat gpurun_out/mmqdiag.log
