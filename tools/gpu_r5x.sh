#!/bin/bash
# Round 5: attention phase stops (KQ_ATTN_DIAG builds) of the unsplit and the split head.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for lib in ${ATTN_LIBS:-adiag adiagsplit}; do
  echo "== $lib"
  MI355X_LIB=ggml-neon-opt_amd/lib/variants/lib$lib.so timeout -k 10 400 python -u tools/attn_phases.py || exit $?
done
