#!/bin/bash
# Round 6: claimed-row decode GEMV (kq_rows_dyn, GEMV_DYN units per wave) against the static
# split (GEMV_DYN=0): the large single GEMVs (bench.large_gemv) and the TinyLlama / Llama-3-8B
# tokens, interleaved. Output: gpurun_out/dyn_ab.txt
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/dyn_ab.txt
: > $OUT
for r in 1 2; do
  for v in 0 default; do
    echo "== large GEMV_DYN=$v (round $r)" >> $OUT
    if [ $v = default ]; then unset MI355X_GEMV_DYN; else export MI355X_GEMV_DYN=$v; fi
    timeout -k 10 150 python -u tools/gemv_large_ab.py 2>&1 | grep -v amdgpu.ids >> $OUT || exit $?
  done
done
unset MI355X_GEMV_DYN
KNOBSETS="- GEMV_DYN=0" timeout -k 10 900 bash tools/knob_ab.sh >> $OUT 2>&1 || exit $?
cat $OUT
