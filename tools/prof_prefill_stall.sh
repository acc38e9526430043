#!/bin/bash
# Round 6: where the prefill GEMM's waves stall. Two PMC passes over
# tools/prefill_bench.py (each within one pass's counter limits: 8 SQ + 1 GRBM), then
# tools/pmc_table.py per kernel. Wait counters are in quad-cycles per wave; the LDS stall
# counters in cycles per SE.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r06}
OUT=gpurun_out/prof_prefill_stall_$TAG
mkdir -p "$OUT"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE \
    --output-format csv -d "$OUT/pass_a" -o run -- python3 tools/prefill_bench.py > "$OUT/pass_a.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_ADDR_CONFLICT SQ_LDS_DATA_FIFO_FULL SQ_INST_CYCLES_VMEM_RD SQ_INSTS_LDS GRBM_GUI_ACTIVE \
    --output-format csv -d "$OUT/pass_b" -o run -- python3 tools/prefill_bench.py > "$OUT/pass_b.log" 2>&1 || exit $?
for p in pass_a pass_b; do
  f=$(find "$OUT/$p" -name "*counter_collection.csv" | head -1)
  echo "== $p"; python3 tools/pmc_table.py "$f" kq_mmq
done | tee "$OUT/summary.md"
