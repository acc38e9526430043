#!/bin/bash
# Round 6: Q6_K prefill tile rows at 240 B (product) vs 224 B (variant q6s224): prefill_bench
# (M = 512, every shape), two interleaved rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
V=$PWD/ggml-neon-opt_amd/lib/variants
OUT=gpurun_out/q6_stride_ab.txt
: > $OUT
for r in 1 2; do
  for L in default q6s224; do
    echo "== $L (round $r)" >> $OUT
    if [ $L = default ]; then unset MI355X_LIB; else export MI355X_LIB=$V/lib$L.so; fi
    PREFILL_TYPES=12,13,14 timeout -k 10 150 python -u tools/prefill_bench.py 2>&1 | grep -v amdgpu.ids >> $OUT || exit $?
  done
done
unset MI355X_LIB
cat $OUT
