#!/bin/bash
# Round 5: instruction-fetch counters of the persistent layer vs the per-node GEMV (two PMC passes).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
P="python3 tools/layer_ab.py --models llama-3-8b --rounds 1 --steps 8"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_IFETCH SQ_INSTS_SALU SQ_INSTS_VALU SQ_BUSY_CYCLES \
  --kernel-include-regex 'kq_layer|kq_rows' -d gpurun_out/r5f_pmc1 -o pmc --output-format csv -- $P > gpurun_out/r5f_pmc1.log 2>&1
rc=$?; echo "pass1 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 300 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS \
  --kernel-include-regex 'kq_layer|kq_rows' -d gpurun_out/r5f_pmc2 -o pmc --output-format csv -- $P > gpurun_out/r5f_pmc2.log 2>&1
rc=$?; echo "pass2 rc=$rc"
find gpurun_out/r5f_pmc1 gpurun_out/r5f_pmc2 -name "*.csv" | head
exit $rc
