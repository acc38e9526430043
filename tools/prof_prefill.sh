#!/bin/bash
# PMC pass of the prefill GEMM (kq_mmq, M = 512): MFMA busy cycles and MFMA
# instruction counts against the kernel's duration (kernel trace in the same run).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r02}
OUT=gpurun_out/prof_prefill_$TAG
mkdir -p "$OUT"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_I8 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
    --output-format csv -d "$OUT/pmc_mfma" -o run -- python3 tools/prefill_bench.py > "$OUT/pmc_mfma.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 tools/prefill_bench.py > "$OUT/trace.log" 2>&1 || exit $?
find "$OUT" -name "*.csv"
