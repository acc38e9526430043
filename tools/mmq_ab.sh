#!/bin/bash
# Prefill GEMM variants (MI355X_MMQ_IMPL = auto / tile64 / k4) on the prefill_bench shapes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; : > gpurun_out/mmq_ab.log
for v in ${VARIANTS:-auto tile64}; do echo "k4 $v" >> gpurun_out/mmq_ab.log; PREFILL_TYPES=${PREFILL_TYPES:-12} MI355X_MMQ_IMPL=$v timeout -k 10 120 python tools/prefill_bench.py >> gpurun_out/mmq_ab.log 2>&1 || exit $?; done
cat gpurun_out/mmq_ab.log
