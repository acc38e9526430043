#!/bin/bash
# PMC passes of the f16 prefill GEMM (kq_mmf, M = 512, Q4_K shapes by default): issue /
# wait breakdown, LDS, L2. Each pass its own run (rocprofv3 does not split counters).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r03}
OUT=gpurun_out/prof_mmf_$TAG
mkdir -p "$OUT"
export MI355X_PREFILL=${MI355X_PREFILL:-f16} PREFILL_TYPES=${PREFILL_TYPES:-12}
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE"
P2="SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_MISC SQ_INSTS_VALU_MFMA_MOPS_F16"
P3="TCC_HIT_sum TCC_MISS_sum FETCH_SIZE"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $P --output-format csv -d "$OUT/p$i" -o run -- \
      python3 tools/prefill_bench.py > "$OUT/p$i.log" 2>&1 || exit $?
  f=$(find "$OUT/p$i" -name "*counter_collection.csv" | head -1)
  python3 tools/pmc_table.py "$f" > "$OUT/p$i.md" && cat "$OUT/p$i.md"
done
