#!/bin/bash
# kq_rows_dyn cost isolation: static split, claimed units, and the dyn kernel with every unit
# static (GEMV_DYN_P=64: no claims), large GEMVs interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/dyn_ab3.txt
: > $OUT
for r in 1 2; do
  for cfg in static claimed; do
    echo "== large $cfg (round $r)" >> $OUT
    unset MI355X_GEMV_DYN MI355X_GEMV_DYN_P
    [ $cfg = static ] && export MI355X_GEMV_DYN=0
    [ $cfg = allstatic ] && export MI355X_GEMV_DYN_P=64
    timeout -k 10 150 python -u tools/gemv_large_ab.py 2>&1 | grep -v amdgpu.ids >> $OUT || exit $?
  done
done
cat $OUT
