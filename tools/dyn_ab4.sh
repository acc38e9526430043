#!/bin/bash
# kq_rows_dyn cost isolation (round 6): static split, claimed units, and the same units dealt
# round-robin without the LDS claim (variant dynrr), large GEMVs interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
V=$PWD/ggml-neon-opt_amd/lib/variants
OUT=gpurun_out/dyn_ab4.txt
: > $OUT
for r in 1 2; do
  for cfg in static claimed rr; do
    echo "== large $cfg (round $r)" >> $OUT
    unset MI355X_GEMV_DYN MI355X_LIB
    [ $cfg = static ] && export MI355X_GEMV_DYN=0
    [ $cfg = rr ] && export MI355X_LIB=$V/libdynrr.so
    timeout -k 10 150 python -u tools/gemv_large_ab.py 2>&1 | grep -v amdgpu.ids >> $OUT || exit $?
  done
done
cat $OUT
